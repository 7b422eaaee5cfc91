"""Per-key limits: a key past the compact tables' 16-bit
fields (more than 65,535 ops, or 16,000 ok returns) is searched by the
32-bit-table path, and register values that span more than one 16-bit state
range are interned per key on the device; neither fails the whole call, and
both agree with the oracle. A key with more distinct values than the state
encoding holds is :unknown on its own (cause "states")."""
import os

import numpy as np
import pytest

from jepsen_amd import _abi as A
from jepsen_amd import synth
from oracle import oracle

pytestmark = pytest.mark.gpu


def _same(v, ov):
    for f in A.VERDICT_FIELDS:
        assert (v[f] == ov[f]).all(), (f, np.nonzero(v[f] != ov[f])[0][:10])


@pytest.mark.parametrize("p_invalid,seed", [(0.0, 7), (1.0, 8)])
def test_long_single_key(ctx, p_invalid, seed):
    """A 200k-op single register (C1 shape, 5 processes): past the compact
    encoding, checked by the 32-bit path; also through jh_check_cas."""
    cols, truth = synth.cas_register(n_keys=1, ops_per_key=200_000, threads_per_key=5, readers=2,
                                     n_values=5, process_limit=5, groups=1, p_info=0.0,
                                     p_invalid=p_invalid, nemesis_every=0, seed=seed)
    assert cols.n > 2 * 65535
    v, s = ctx.check_cas_independent(cols)
    ov, _ = oracle.check_cas_independent(cols, threads=1)
    _same(v, ov)
    assert int(v["valid"][0]) == (A.INVALID if truth[0] else A.VALID)


def test_long_keys_beside_short(ctx):
    """Long keys and ordinary keys in one call: each takes its own path."""
    from jepsen_amd.history import Columns
    a, _ = synth.cas_register(n_keys=2, ops_per_key=40_000, threads_per_key=5, readers=2, process_limit=5,
                              groups=2, p_info=0.0, p_invalid=0.5, nemesis_every=0, seed=11)
    b, _ = synth.cas_register(n_keys=200, ops_per_key=300, seed=12)
    key = np.concatenate([a.key, np.where(b.key >= 0, b.key + 2, -1)])
    proc = np.concatenate([a.process, np.where(b.process >= 0, b.process + 1000, b.process)])
    cols = Columns(n=a.n + b.n, process=proc, type=np.concatenate([a.type, b.type]),
                   f=np.concatenate([a.f, b.f]), key=key, value=np.concatenate([a.value, b.value]),
                   value2=np.concatenate([a.value2, b.value2]), n_keys=202, aux=np.zeros(1, np.int64))
    v, s = ctx.check_cas_independent(cols)
    ov, _ = oracle.check_cas_independent(cols, threads=8)
    _same(v, ov)


@pytest.mark.parametrize("init", [None, 0, 123456789])
def test_unique_values(ctx, init):
    """Values drawn from 0..1e9: one global span is far too wide, so the
    device numbers each key's values densely (with the initial value first)."""
    cols, _ = synth.cas_register(n_keys=300, ops_per_key=300, n_values=1_000_000_000, p_invalid=0.05,
                                 init_nil=init is None, seed=9)
    if init not in (None, 0):
        # the generator's (cas-register 0) start as another value: shift every 0
        for c in (cols.value, cols.value2):
            c[c == 0] = init
    v, s = ctx.check_cas_independent(cols, init=init)
    ov, _ = oracle.check_cas_independent(cols, init=A.NIL if init is None else init, threads=8)
    _same(v, ov)
    assert (v["valid"] == A.INVALID).sum() > 0


def test_per_key_interning_forced(ctx):
    """JH_LIN_INTERN_PER_KEY takes the per-key path on an ordinary C3 slice:
    same verdicts and counts as the global numbering and the oracle."""
    cols, _ = synth.cas_register(n_keys=1000, ops_per_key=500, p_invalid=0.02, seed=13)
    v0, s0 = ctx.check_cas_independent(cols)
    v1, s1 = ctx.check_cas_independent(cols, flags=A.LIN_INTERN_PER_KEY)
    assert (v0 == v1).all()
    ov, _ = oracle.check_cas_independent(cols, threads=8)
    _same(v1, ov)


def test_too_many_states_is_per_key(ctx):
    """One key writes 70k distinct values (beyond the 16-bit states): that key
    is :unknown with cause "states"; the others are checked as usual."""
    from jepsen_amd.history import Columns
    a, _ = synth.cas_register(n_keys=1, ops_per_key=150_000, threads_per_key=5, readers=2, process_limit=5,
                              groups=1, n_values=1_000_000_000, p_info=0.0, p_invalid=0.0, nemesis_every=0,
                              seed=14)
    b, _ = synth.cas_register(n_keys=50, ops_per_key=300, seed=15)
    key = np.concatenate([a.key, np.where(b.key >= 0, b.key + 1, -1)])
    proc = np.concatenate([a.process, np.where(b.process >= 0, b.process + 1000, b.process)])
    cols = Columns(n=a.n + b.n, process=proc, type=np.concatenate([a.type, b.type]),
                   f=np.concatenate([a.f, b.f]), key=key, value=np.concatenate([a.value, b.value]),
                   value2=np.concatenate([a.value2, b.value2]), n_keys=51, aux=np.zeros(1, np.int64))
    assert len(np.unique(a.value[a.value != A.NIL])) > 65535
    v, s = ctx.check_cas_independent(cols)
    assert int(v["valid"][0]) == A.UNKNOWN and A.CAUSES[int(v["cause"][0])] == "states"
    ov, _ = oracle.check_cas_independent(cols, threads=8)
    _same(v[1:], ov[1:])


def test_huge_budget_fits_memory():
    """the phase-2/3 memo tables, the WIDE pipeline and
    the BFS workgroups are sized for the full budget, so at 2^24 they would
    ask for more than the device holds; every such table is clamped by free
    HBM (fit_units), and the call still returns every verdict, equal to the
    oracle's. A private context: its tables are freed afterwards."""
    from jepsen_amd import _native
    cols, _ = synth.cas_register(n_keys=300, ops_per_key=600, p_invalid=0.05, p_info=0.03, seed=131)
    c, _ = oracle.check_cas_independent(cols, budget=1 << 24, threads=16)
    ctx = _native.Context(0)
    try:
        g, s = ctx.check_cas_independent(cols, budget=1 << 24, quick_budget=200)
    finally:
        ctx.close()
    for f in A.VERDICT_FIELDS:
        assert (g[f] == c[f]).all(), f
    assert s.n_deferred > 0
