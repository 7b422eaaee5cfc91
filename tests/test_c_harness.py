"""The C ABI as a non-Python caller sees it: tests/c/jh_harness.c links
libjh.so with gcc and calls it with plain pointers (what the JNA shim of
INTEGRATION.md does). CPU tests: the ABI version, jh_open's error code without
a device, and jh_key_costs against a Python restatement of the window-sum
estimate. GPU tests: jh_check_cas_independent through the harness, on one
context and on a multi-device context (jh_open_devices with the same device
three times, which drives the split / per-device check / merge path of
jh_multi.hip on one GPU), against the oracle."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "tests", "c", "jh_harness")


def _write(cols, path):
    with open(path, "wb") as fh:
        np.array([cols.n, cols.n_keys], np.int64).tofile(fh)
        for c in ("process", "type", "f", "key", "value", "value2"):
            np.ascontiguousarray(getattr(cols, c), dtype=np.int64).tofile(fh)


def _run(*args):
    r = subprocess.run([EXE, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def _costs_py(cols):
    """Window-sum restatement: per key, entries + sum over client ops of the
    :ok returns inside the op's window (a crashed op's window runs to the end)."""
    K = cols.n_keys
    ent = np.zeros(K, np.int64)
    nok = np.zeros(K, np.int64)
    acc = np.zeros(K, np.int64)
    ncr = np.zeros(K, np.int64)
    for i in range(cols.n):
        k = int(cols.key[i])
        if k < 0 or k >= K or cols.process[i] < 0:
            continue
        t = int(cols.type[i])
        ent[k] += 1
        if t == 0:
            acc[k] -= nok[k]
        elif t == 1:
            nok[k] += 1
            acc[k] += nok[k]
        elif t == 2:
            acc[k] += nok[k]
        elif t == 3:
            ncr[k] += 1
    return ent + np.maximum(0, acc + ncr * nok)


def _hist(n_keys, seed, **kw):
    from jepsen_amd import synth
    g = dict(threads_per_key=10, readers=5, n_values=5, process_limit=20, groups=10, init_nil=True,
             p_info=0.02, p_invalid=0.05, nemesis_every=3000)
    g.update(kw)
    return synth.cas_register(n_keys=n_keys, ops_per_key=200, seed=seed, **g)[0]


def test_version(built):
    from jepsen_amd import _abi as A
    assert int(_run("version")) == A.JH_ABI_VERSION


def test_open_without_device(built):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a device is present")
    from jepsen_amd import _abi as A
    assert int(_run("open")) == A.JH_EDEVICE


@pytest.mark.parametrize("seed", [1, 2])
def test_key_costs(built, tmp_path, seed):
    from jepsen_amd import shard
    cols = _hist(60, seed, p_info=0.1)
    _write(cols, tmp_path / "h.bin")
    _run("costs", str(tmp_path / "h.bin"), str(tmp_path / "c.bin"))
    got = np.fromfile(tmp_path / "c.bin", np.int64)
    exp = _costs_py(cols)
    assert (got == exp).all()
    assert (shard.key_costs(cols) == exp).all()


def test_key_costs_edges(built, tmp_path):
    from jepsen_amd.history import Columns
    z = np.zeros(0, np.int64)
    empty = Columns(n=0, process=z, type=z, f=z, key=z, value=z, value2=z, n_keys=3, aux=np.zeros(1, np.int64))
    _write(empty, tmp_path / "e.bin")
    _run("costs", str(tmp_path / "e.bin"), str(tmp_path / "c.bin"))
    assert (np.fromfile(tmp_path / "c.bin", np.int64) == 0).all()


def _check_vs_oracle(tmp_path, cols, devs=None, quick=None):
    from jepsen_amd import _abi as A
    from oracle import oracle
    _write(cols, tmp_path / "h.bin")
    args = ["check", str(tmp_path / "h.bin"), str(tmp_path / "v.bin")] + ([devs] if devs else [])
    if quick:
        args.append(str(quick))
    out = _run(*args)
    got = np.fromfile(tmp_path / "v.bin", dtype=A.VERDICT_DTYPE)
    ov, os_ = oracle.check_cas_independent(cols, threads=8)
    for f in A.VERDICT_FIELDS:
        assert (got[f] == ov[f]).all(), f
    summ = dict(kv.split("=") for kv in out.split("\n")[1].split())
    ff = ov["fail_entry"][ov["valid"] == A.INVALID]
    assert int(summ["first_fail_entry"]) == (int(ff.min()) if len(ff) else -1)
    assert int(summ["n_invalid"]) == int((ov["valid"] == A.INVALID).sum())
    assert int(summ["explored"]) == int(ov["explored"][ov["explored"] > 0].sum())
    return out


@pytest.mark.gpu
def test_check_single_device(built, tmp_path):
    out = _check_vs_oracle(tmp_path, _hist(300, 11))
    assert out.startswith("devices=1")


@pytest.mark.gpu
@pytest.mark.parametrize("devs", ["0,0", "0,0,0"])
def test_check_multi_context(built, tmp_path, devs):
    out = _check_vs_oracle(tmp_path, _hist(300, 12), devs)
    assert out.startswith(f"devices={len(devs.split(','))}")


@pytest.mark.gpu
@pytest.mark.parametrize("devs", ["0,0", "0,0,0,0"])
def test_multi_context_pooled_heavy_keys(built, tmp_path, devs):
    """jh_open_devices checks in two stages -- phase 1 on
    each device's cost-model share, then the deferred keys of every device
    pooled and pulled by the member threads in batches (guided
    self-scheduling). With a small quick budget most keys take the second
    stage; every verdict field still equals the oracle's."""
    cols = _hist(400, 17)
    out = _check_vs_oracle(tmp_path, cols, devs, quick=40)
    summ = dict(kv.split("=") for kv in out.split("\n")[1].split())
    assert int(summ["n_deferred"]) > 50


@pytest.mark.gpu
def test_multi_context_pools_wide_window_keys(built, tmp_path):
    """stage 1 of the two-stage check hands the 65-256-member
    keys back deferred too (they are the heaviest), so stage 2 pools them
    with the rest. C5-shaped keys (50 threads per key, many :info) on two
    contexts: several windows over 64 members, every verdict field equal to
    the oracle's."""
    from jepsen_amd import synth
    cols = synth.cas_register(n_keys=24, ops_per_key=160, threads_per_key=50, readers=25, n_values=5,
                              process_limit=100, groups=10, init_nil=True, p_info=0.2, p_invalid=0.05,
                              nemesis_every=10000, seed=23)[0]
    from jepsen_amd import _abi as A
    wide = 0
    for k in range(cols.n_keys):
        t = cols.type[cols.key == k]
        opened = np.cumsum(np.where(t == A.TYPE_INVOKE, 1, np.where((t == A.TYPE_OK) | (t == A.TYPE_FAIL), -1, 0)))
        wide += int(opened.max() > 64)
    assert wide >= 2
    _check_vs_oracle(tmp_path, cols, "0,0")
