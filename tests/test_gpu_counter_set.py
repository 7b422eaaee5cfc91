"""Parity of the device counter and set checkers with the oracle and with the
reference's known answers (checker_test.clj:90-166)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLD, load_npz_cols
from jepsen_amd import _abi as A
from jepsen_amd import checker
from jepsen_amd import history as H
from jepsen_amd import synth
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLD, "counter.json")))["cases"],
                         ids=lambda c: c["name"])
def test_counter_known_answers_device(ctx, case):
    r = checker.check(checker.counter(), None, case["history"], {})
    assert r == case["expected"]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_counter_random(ctx, seed):
    cols = synth.counter(n_ops=200000, n_procs=10 + seed, read_every=11, p_fail=0.05, p_info=0.02,
                         n_bad_reads=3 * seed, seed=seed)
    g = ctx.check_counter(cols)
    c = oracle.check_counter(cols)
    assert g["valid"] == c["valid"] and g["cause"] == c["cause"]
    assert g["n_reads"] == c["n_reads"] and g["n_errors"] == c["n_errors"]
    assert g["first_err_entry"] == c["first_err_entry"]
    assert (g["reads"] == c["reads"]).all()


def test_counter_golden(ctx):
    cols, z = load_npz_cols("synthetic_counter.npz")
    g = ctx.check_counter(cols)
    assert (g["reads"] == z["reads"]).all() and g["valid"] == int(z["valid"])
    assert g["first_err_entry"] == int(z["first_err_entry"])


def test_counter_c2_scale(ctx):
    """C2 counter: 100M entries, add:read 100:1 -- device result must be
    self-consistent (reads non-decreasing bounds) and the valid variant valid."""
    cols = synth.counter(n_ops=50_000_000, n_procs=10, read_every=101, p_fail=0.05, p_info=0.01,
                         n_bad_reads=0, seed=2)
    g = ctx.check_counter(cols, reads_cap=1 << 22)
    assert g["valid"] == A.VALID and g["n_errors"] == 0
    r = g["reads"]
    assert (r[:, 0] <= r[:, 1]).all() and (r[:, 1] <= r[:, 2]).all()


def test_counter_errors(ctx):
    inv = lambda p, f, v: {"process": p, "type": "invoke", "f": f, "value": v}
    ok = lambda p, f, v: {"process": p, "type": "ok", "f": f, "value": v}
    for h in ([inv(0, "add", 1), inv(0, "add", 1)], [ok(0, "add", 1)],
              [inv(0, "add", None), ok(0, "add", None)],
              [inv(0, "read", None), ok(0, "read", None)]):
        cols = H.encode(h, keyed=False)
        g = ctx.check_counter(cols)
        c = oracle.check_counter(cols)
        assert (g["valid"], g["cause"]) == (c["valid"], c["cause"]) and g["valid"] == A.UNKNOWN


def _counter_same(g, c):
    assert (g["valid"], g["cause"]) == (c["valid"], c["cause"])
    assert g["n_reads"] == c["n_reads"] and g["n_errors"] == c["n_errors"]
    assert g["first_err_entry"] == c["first_err_entry"]
    if c["n_reads"]:
        assert (g["reads"] == c["reads"]).all()


@pytest.mark.parametrize("n_procs", [4, 40])
@pytest.mark.parametrize("at", [2040, 2047, 4095])
def test_counter_mismatched_completion_across_chunks(ctx, n_procs, at):
    """an [:invoke :add] whose completion is an [:ok :read]
    in a later 2048-row chunk (the pack spills it), or of a process past the
    chunk's 32 tracked ones, is an orphan read exactly as inside one chunk --
    the verdict may not depend on where the chunk boundaries fall."""
    inv = lambda p, f, v: {"process": p, "type": "invoke", "f": f, "value": v}
    ok = lambda p, f, v: {"process": p, "type": "ok", "f": f, "value": v}
    h, total, p = [], 0, 0
    while len(h) < at:
        q = 1 + (p % (n_procs - 1))        # processes 1..n_procs-1 as filler
        h += [inv(q, "add", 1), ok(q, "add", 1)]
        total += 1
        p += 1
        if p % 50 == 0:
            h += [inv(q, "read", None), ok(q, "read", total)]
    h = h[:at]
    if len(h) % 2:
        h.pop()
    h.append(inv(0, "add", 1))                      # process 0's invocation ...
    for k in range(12):                             # ... past the chunk boundary
        q = 1 + (k % (n_procs - 1))
        h += [inv(q, "add", 1), ok(q, "add", 1)]
    h.append(ok(0, "read", 5))                      # ... completed by a read
    h += [inv(1, "read", None), ok(1, "read", 7)]
    cols = H.encode(h, keyed=False)
    _counter_same(ctx.check_counter(cols), oracle.check_counter(cols))


def test_counter_many_processes_random(ctx):
    """More than the pack's 32 tracked processes per chunk, with :info and
    :fail completions, against the oracle."""
    cols = synth.counter(n_ops=300000, n_procs=90, read_every=7, p_fail=0.05, p_info=0.02,
                         n_bad_reads=5, seed=11)
    _counter_same(ctx.check_counter(cols), oracle.check_counter(cols))


def _set_same(g, c):
    for k in ("valid", "cause", "attempt_count", "acknowledged_count", "ok_count", "lost_count",
              "recovered_count", "unexpected_count", "first_fail_entry", "final_read_entry"):
        assert g[k] == c[k], k
    for i in range(4):
        assert g["n_runs"][i] == c["n_runs"][i]
        assert (g["runs"][i] == c["runs"][i]).all(), i


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_set_random(ctx, seed):
    cols = synth.set_history(n_adds=300000, n_procs=10, p_fail=0.05, p_info=0.03,
                             n_lost=seed * 7, n_unexpected=seed, seed=seed)
    c = oracle.check_set(cols)
    _set_same(ctx.check_set(cols), c)
    _bits_same(ctx.check_set_bitmaps(cols), c)


def _bits_same(b, c):
    """jh_check_set_bitmaps against the oracle: counts, rows, and every run."""
    from jepsen_amd._native import bits_to_runs
    for k in ("valid", "cause", "attempt_count", "acknowledged_count", "ok_count", "lost_count",
              "recovered_count", "unexpected_count", "first_fail_entry", "final_read_entry"):
        assert b[k] == c[k], k
    if b["valid"] == A.UNKNOWN:
        return
    for i in range(4):
        r = bits_to_runs(b["bits"][i], b["base"])
        assert b["n_runs"][i] == c["n_runs"][i] and len(r) == c["n_runs"][i], i
        assert (r == np.asarray(c["runs"][i]).reshape(-1, 2)).all(), i


def test_set_golden_and_map(ctx):
    cols, z = load_npz_cols("synthetic_set.npz")
    g = ctx.check_set(cols)
    assert g["valid"] == int(z["valid"]) and g["first_fail_entry"] == int(z["first_fail_entry"])
    assert (g["runs"][1] == z["runs_lost"]).all()
    r = checker.SetChecker().check(None, cols, {})
    assert r["lost-count"] == int(z["counts"][3])
    assert r["lost"] == checker._runs_str(z["runs_lost"].tolist())


def test_set_edge_cases(ctx):
    inv = lambda p, f, v: {"process": p, "type": "invoke", "f": f, "value": v}
    ok = lambda p, f, v: {"process": p, "type": "ok", "f": f, "value": v}
    # never read
    r = checker.check(checker.set(), None, [inv(0, "add", 1), ok(0, "add", 1)], {})
    assert r == {"valid?": "unknown", "error": "Set was never read"}
    # reads: the LAST ok read counts; elements in any order
    h = [inv(0, "add", 1), ok(0, "add", 1), inv(0, "add", 2), ok(0, "add", 2),
         inv(1, "read", None), ok(1, "read", [5]),
         inv(1, "read", None), ok(1, "read", [2, 1, 9])]
    r = checker.check(checker.set(), None, h, {})
    assert r["valid?"] is False and r["unexpected"] == "#{9}" and r["ok"] == "#{1..2}"
    assert r["lost"] == "#{}" and r["recovered-count"] == 0
    cols = H.encode(h, keyed=False)
    c = oracle.check_set(cols)
    _set_same(ctx.check_set(cols), c)
    _bits_same(ctx.check_set_bitmaps(cols), c)


def test_counter_many_procs(ctx):
    """More processes than a chunk's compact pairing index (32): their
    invocations take the spill walk from the next row; heavy :info makes many
    walks start at the chunk's end (crashed ops, retired processes)."""
    cols = synth.counter(n_ops=300000, n_procs=300, read_every=11, p_fail=0.05, p_info=0.1,
                         n_bad_reads=5, seed=9)
    g = ctx.check_counter(cols)
    c = oracle.check_counter(cols)
    assert (g["valid"], g["cause"], g["n_reads"], g["n_errors"], g["first_err_entry"]) == \
        (c["valid"], c["cause"], c["n_reads"], c["n_errors"], c["first_err_entry"])
    assert (g["reads"] == c["reads"]).all()


def test_counter_host_buffer(ctx):
    """Triples into a reused page-locked buffer (jh_host_alloc): same result."""
    from jepsen_amd._native import HostBuffer
    cols = synth.counter(n_ops=100000, n_procs=10, read_every=11, p_fail=0.05, p_info=0.02,
                         n_bad_reads=2, seed=4)
    hb = HostBuffer(3 * int(cols.n), np.int64)
    c = oracle.check_counter(cols)
    for _ in range(2):
        g = ctx.check_counter(cols, out=hb.array)
        assert (g["reads"] == c["reads"]).all() and g["n_errors"] == c["n_errors"]


from hipcols import DevCols as _DevCols  # noqa: E402


@pytest.mark.parametrize("shift", [0, 1])
def test_set_device_columns_alignment(ctx, shift):
    """Device-resident columns 16-byte aligned (row pairs in one load) and only
    8-byte aligned (two loads per pair): same result as the oracle."""
    cols = synth.set_history(n_adds=200001, n_procs=10, p_fail=0.05, p_info=0.03,
                             n_lost=5, n_unexpected=2, seed=11)
    c = oracle.check_set(cols)
    d = _DevCols(cols, shift)
    _bits_same(ctx.check_set_bitmaps(d, words_cap=1 << 16, on_device=True), c)
    _set_same(ctx.check_set(d, runs_cap=int(cols.n) + 8, on_device=True), c)


def test_set_sparse_span(ctx):
    """Elements spread over a span far wider than the history: the direct
    bitmap path (no byte maps, no buckets)."""
    inv = lambda p, f, v: {"process": p, "type": "invoke", "f": f, "value": v}
    ok = lambda p, f, v: {"process": p, "type": "ok", "f": f, "value": v}
    h, els = [], []
    for i in range(400):
        v = i * 100_003 if i % 2 else -i * 77_777
        h += [inv(i % 5, "add", v), ok(i % 5, "add", v)]
        if i % 9:
            els.append(v)
    els.append(5)                       # never attempted: unexpected
    rng = np.random.default_rng(3)
    rng.shuffle(els)
    h += [inv(7, "read", None), ok(7, "read", [int(x) for x in els])]
    cols = H.encode(h, keyed=False)
    c = oracle.check_set(cols)
    _set_same(ctx.check_set(cols), c)
    _bits_same(ctx.check_set_bitmaps(cols, words_cap=1 << 22), c)


@pytest.mark.parametrize("n_procs", [6, 40])
@pytest.mark.parametrize("tail", ["ok", "info-then-ok", "fail", "double-invoke", "crash"])
def test_counter_walk_across_chunks(ctx, n_procs, tail):
    """A spilled invocation whose process is silent for several 2048-row
    chunks: k_cnt_pair_spill jumps chunk to chunk on their first-row tables
    (or walks chunks with more than 32 processes), past :info rows of the
    process, to the completion, a double invocation, or nothing (a crash)."""
    inv = lambda p, f, v: {"process": p, "type": "invoke", "f": f, "value": v}
    ok = lambda p, f, v: {"process": p, "type": "ok", "f": f, "value": v}

    def filler(h, rows, k0):
        for k in range(rows // 2):
            q = 1 + ((k0 + k) % (n_procs - 1))
            h += [inv(q, "add", 1), ok(q, "add", 1)]
    h = []
    filler(h, 1500, 0)
    h.append(inv(0, "add", 3))                       # process 0's invocation in chunk 0
    filler(h, 5000, 7)                               # chunks 1 and 2: no row of process 0
    if tail == "info-then-ok":
        h.append({"process": 0, "type": "info", "f": "add", "value": 3})
        filler(h, 900, 3)
    if tail in ("ok", "info-then-ok"):
        h.append(ok(0, "add", 3))
    elif tail == "fail":
        h.append({"process": 0, "type": "fail", "f": "add", "value": 3})
    elif tail == "double-invoke":
        h.append(inv(0, "add", 1))
    filler(h, 300, 5)
    h += [inv(1, "read", None), ok(1, "read", 7)]
    cols = H.encode(h, keyed=False)
    _counter_same(ctx.check_counter(cols), oracle.check_counter(cols))
