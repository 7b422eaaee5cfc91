"""Parity of the device linearizability path (libjh.so, through the C ABI)
with the CPU oracle: verdict, cause, first failing row and WGL cache size
must be bit-identical on every key."""
import json
import os

import numpy as np
import pytest

from conftest import GOLD, load_npz_cols
from jepsen_amd import _abi as A
from jepsen_amd import history as H
from jepsen_amd import synth
from oracle import oracle

pytestmark = pytest.mark.gpu


def _same(gpu, cpu):
    """Verdict, cause, failing row and WGL's cache size, key by key (explored
    is exact and deterministic on every key: include/jh.h)."""
    for f in A.VERDICT_FIELDS:
        bad = np.nonzero(gpu[f] != cpu[f])[0]
        assert len(bad) == 0, (f, bad[:10], gpu[bad[:5]], cpu[bad[:5]])


def test_perf_test_history(ctx):
    d = json.load(open(os.path.join(GOLD, "perf_test.json")))
    cols = H.encode(d["history"], keyed=False)
    g = ctx.check_cas(cols, init=0)
    c = oracle.check_cas(cols, init=0)
    assert g[0] == A.VALID and tuple(g) == tuple(c)
    g = ctx.check_cas(cols, init=None)
    c = oracle.check_cas(cols, init=A.NIL)
    assert g[0] == A.INVALID and tuple(g) == tuple(c)


@pytest.mark.parametrize("name", ["cas_small", "cas_tiny", "cas_init0", "cas_crashy"])
def test_golden_vectors(ctx, name):
    man = {m["name"]: m for m in json.load(open(os.path.join(GOLD, "manifest.json")))["synthetic"]}
    cols, z = load_npz_cols(f"synthetic_{name}.npz")
    v, s = ctx.check_cas_independent(cols, init=man[name]["init"])
    exp = np.zeros(cols.n_keys, A.VERDICT_DTYPE)
    for f in ("valid", "cause", "fail_entry", "explored"):
        exp[f] = z[f]
    for f in ("valid", "cause", "fail_entry", "explored"):
        bad = np.nonzero(v[f] != exp[f])[0]
        assert len(bad) == 0, (f, bad[:10])
    assert s.n_invalid == man[name]["n_invalid"]


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_random_histories(ctx, seed):
    cols, _ = synth.cas_register(n_keys=500, ops_per_key=120, threads_per_key=8, readers=3,
                                 groups=8, p_info=0.05, p_invalid=0.05, seed=1000 + seed)
    g, gs = ctx.check_cas_independent(cols)
    c, cs = oracle.check_cas_independent(cols, threads=8)
    _same(g, c)
    assert (gs.valid, gs.n_invalid, gs.n_unknown, gs.first_fail_entry, gs.explored) == \
           (cs.valid, cs.n_invalid, cs.n_unknown, cs.first_fail_entry, cs.explored)


def test_budget_and_deferral(ctx):
    """Keys past the quick budget go to the deep pass; keys past the full
    budget are :unknown with explored == budget, exactly like the oracle."""
    cols, _ = synth.cas_register(n_keys=300, ops_per_key=300, p_invalid=0.2, seed=77)
    for budget in (100, 3000, 50000):
        g, _ = ctx.check_cas_independent(cols, budget=budget)
        c, _ = oracle.check_cas_independent(cols, budget=budget, threads=8)
        _same(g, c)


@pytest.mark.parametrize("quick", [1, 40, 700])
def test_heavy_key_paths(ctx, quick):
    """Force keys through the deferral -> workgroup BFS -> sequential DFS
    cascade with a tiny quick budget: results must not change."""
    cols, _ = synth.cas_register(n_keys=400, ops_per_key=150, p_invalid=0.2, p_info=0.05, seed=88)
    c, _ = oracle.check_cas_independent(cols, threads=8)
    g, _ = ctx.check_cas_independent(cols, quick_budget=quick)
    _same(g, c)
    g, _ = ctx.check_cas_independent(cols, budget=2000, quick_budget=quick)
    c, _ = oracle.check_cas_independent(cols, budget=2000, threads=8)
    _same(g, c)


NOW = A.LIN_HELPERS_NOW


@pytest.mark.parametrize("tune", [
    dict(flags=NOW, quick_budget=40),
    dict(flags=NOW, quick_budget=40, helpers=48),
    dict(flags=NOW, quick_budget=40, phase2_budget=300, lean_waves=8),
    dict(flags=NOW, quick_budget=40, p2_waves_per_cu=1),
    dict(flags=A.LIN_NO_HELPERS, quick_budget=40),
    dict(p1_waves_per_cu=1, quick_budget=500, handover_min=100),
])
def test_late_helpers(ctx, tune):
    """Phase-2 late helpers (the workgroup engine racing the sequential search
    and the BFS on long-running keys): with no delay every deferred key gets a
    helper, which settles some of them first, hands others back when phase 3
    takes the key (small phase-2 budget), or loses the race. Every verdict,
    cause, failing row and WGL count must equal the oracle's, at the full
    budget and at a budget the helpers run into."""
    cols, _ = synth.cas_register(n_keys=400, ops_per_key=200, p_invalid=0.1, p_info=0.05, seed=95)
    for budget in (None, 3000):
        g, _ = ctx.check_cas_independent(cols, budget=budget, **tune)
        c, _ = oracle.check_cas_independent(cols, budget=budget or A.DEFAULT_BUDGET, threads=8)
        _same(g, c)


@pytest.mark.parametrize("p2,waves", [(4097, 1), (4097, 6), (9000, 3)])
def test_phase3_handover(ctx, p2, waves):
    """With fewer phase-2 waves than deferred keys, keys past the phase-2
    budget restart in phase 3 (on phase 2's tables, the kernel picked on the
    device by phase 3's key count: one wave per CU for few keys, four for
    many): a small phase-2 budget and few waves must not change any result,
    with the full budget or a budget in between."""
    cols, _ = synth.cas_register(n_keys=300, ops_per_key=400, p_invalid=0.1, p_info=0.05, seed=91)
    for budget in (None, 20000):
        g, s = ctx.check_cas_independent(cols, budget=budget, phase2_budget=p2, lean_waves=waves, quick_budget=500)
        c, _ = oracle.check_cas_independent(cols, budget=budget or A.DEFAULT_BUDGET, threads=8)
        _same(g, c)
        assert s.waves[0] == min(waves, s.n_deferred - s.n_deferred_wide)
    assert s.n_phase3 > 0


@pytest.mark.parametrize("handover", [64, 1024, -1])
def test_phase1_handover(ctx, handover):
    """Phase 1 hands a search past handover_min inserts to the heavy-key pass
    once its queue is empty (the pass restarts it with the full budget): the
    hand-over only moves keys between phases, so verdicts, causes, failing
    rows and WGL counts equal the oracle's at two budgets, and a lower
    threshold defers at least as many keys as none (-1)."""
    cols, _ = synth.cas_register(n_keys=600, ops_per_key=300, p_invalid=0.1, p_info=0.05, seed=97)
    for budget in (None, 5000):
        g, s = ctx.check_cas_independent(cols, budget=budget, quick_budget=4000, handover_min=handover)
        c, _ = oracle.check_cas_independent(cols, budget=budget or A.DEFAULT_BUDGET, threads=8)
        _same(g, c)
        _, s0 = ctx.check_cas_independent(cols, budget=budget, quick_budget=4000, flags=A.LIN_NO_HANDOVER)
        assert s.n_deferred >= s0.n_deferred


@pytest.mark.parametrize("quick,handover", [(300, 0), (2000, 0), (8192, 0), (2000, 256)])
def test_resume_deferred(ctx, quick, handover):
    """Round 5: phase 1 saves every deferred LEAN search -- its stack and its
    memo, WGL's cache -- and the heavy-key pass continues it instead of
    restarting. Continued and restarted (JH_LIN_NO_RESUME) searches give every
    field equal to the oracle's, at the full budget and at one the continued
    searches run into; records were saved and used."""
    cols, _ = synth.cas_register(n_keys=400, ops_per_key=600, threads_per_key=10, readers=5, p_invalid=0.05,
                                 p_info=0.03, seed=98)
    for budget in (None, 20000):
        c, _ = oracle.check_cas_independent(cols, budget=budget or A.DEFAULT_BUDGET, threads=16)
        g, s = ctx.check_cas_independent(cols, budget=budget, quick_budget=quick, handover_min=handover)
        _same(g, c)
        g2, s2 = ctx.check_cas_independent(cols, budget=budget, quick_budget=quick, handover_min=handover,
                                           flags=A.LIN_NO_RESUME)
        _same(g2, c)
        assert s.resumed > 0 and s2.resumed == 0 and s.resume_bytes > 0
        assert s.resumed <= s.n_deferred


@pytest.mark.parametrize("waves", [None, 1])
def test_windows_wider_than_64(ctx, waves):
    """Windows of 65..256 members (k_lin_xw, 4-word masks) and wider than
    256 (:unknown, cause window): verdict, cause, failing row and WGL cache
    size equal the oracle's at several budgets; one wave (xw_waves=1)
    checks every wide key in turn with the same HBM table."""
    tune = {"xw_waves": waves} if waves else {}
    cols, _ = synth.cas_register(n_keys=24, ops_per_key=260, threads_per_key=120, readers=20,
                                 groups=120, process_limit=10 ** 6, p_info=0.08, p_invalid=0.2,
                                 seed=61)
    for budget in (3000, 40000) if waves else (3000, 40000, None):
        g, _ = ctx.check_cas_independent(cols, budget=budget, **tune)
        c, _ = oracle.check_cas_independent(cols, budget=budget or A.DEFAULT_BUDGET, threads=16)
        _same(g, c)
    assert (c["cause"] != 2).sum() > 0


def test_c5_shape(ctx):
    """C5-shaped keys (50 threads per key, 20% :info): deep searches that
    mostly end :unknown at the full budget (phase 3, HBM memo at full load),
    windows over 64, a few settled keys; identical to the oracle."""
    cols, _ = synth.cas_register(n_keys=24, ops_per_key=500, threads_per_key=50, readers=25,
                                 process_limit=100, p_info=0.2, p_invalid=0.05, seed=5)
    g, gs = ctx.check_cas_independent(cols)
    c, cs = oracle.check_cas_independent(cols, threads=16)
    _same(g, c)
    assert gs.n_unknown == cs.n_unknown and gs.n_unknown > 0


@pytest.mark.parametrize("tune", [dict(), dict(wide_waves=2, phase2_budget=3000), dict(wide_waves=5)])
def test_wide_pipeline(ctx, tune):
    """The deferred WIDE keys (windows of 41-64 members) on their own stream:
    a wave per key and one pass at the full budget (default), or fewer waves
    than keys -- phase 2 to phase2_budget, then phase 3 restarts the keys past
    it on the same tables, its key count read on the device. Verdicts, causes,
    failing rows and WGL counts equal the oracle's at two budgets."""
    cols, _ = synth.cas_register(n_keys=40, ops_per_key=300, threads_per_key=50, readers=25,
                                 process_limit=100, p_info=0.1, p_invalid=0.1, seed=71)
    for budget in (40000, 200000):
        g, gs = ctx.check_cas_independent(cols, budget=budget, quick_budget=300, **tune)
        c, _ = oracle.check_cas_independent(cols, budget=budget, threads=16)
        _same(g, c)
        assert gs.n_deferred_wide > 0 and gs.waves[1] == min(gs.n_deferred_wide, tune.get("wide_waves", 1 << 30))
        assert gs.wide_entries > 0 and gs.wide_ms > 0
    if "phase2_budget" in tune:
        assert gs.n_phase3_wide > 0


def test_c3_scale_properties(ctx):
    """BASELINE config C3 (10k keys x ~1k entries): every key the generator
    did not fault is valid, and the device equals the oracle on every key."""
    cols, truth = synth.cas_register(seed=3)
    g, gs = ctx.check_cas_independent(cols)
    assert not ((g["valid"] == A.INVALID) & (truth == 0)).any()
    assert gs.n_keys == cols.n_keys
    c, cs = oracle.check_cas_independent(cols, threads=16)
    _same(g, c)


def test_single_key_c1(ctx):
    """C1: one key, 5 processes, 10k entries (plain history, no tuples)."""
    cols, _ = synth.cas_register(n_keys=1, ops_per_key=5000, threads_per_key=5, readers=2,
                                 groups=1, p_info=0.01, p_invalid=0.0, seed=1, keyed=False,
                                 process_limit=10 ** 6)
    g = ctx.check_cas(cols)
    c = oracle.check_cas(cols)
    assert tuple(g) == tuple(c) and g[0] == A.VALID


def test_edge_cases(ctx):
    inv = lambda p, f, v: {"process": p, "type": "invoke", "f": f, "value": v}
    ok = lambda p, f, v: {"process": p, "type": "ok", "f": f, "value": v}
    info = lambda p, f, v: {"process": p, "type": "info", "f": f, "value": v}
    fail = lambda p, f, v: {"process": p, "type": "fail", "f": f, "value": v}
    cases = [
        [],
        [{"process": "nemesis", "type": "info", "f": "start"}],
        [inv(0, "write", 1), inv(0, "write", 2)],
        [inv(0, "write", 1), info(0, "write", 1), inv(0, "write", 2)],
        [ok(0, "write", 1)],
        [inv(0, "incr", 1), ok(0, "incr", 1)],
        [inv(0, "incr", 1), fail(0, "incr", 1)],
        [inv(0, "write", 3), info(0, "write", 3), inv(1, "read", None), ok(1, "read", 3)],
        [inv(0, "cas", [None, 2]), ok(0, "cas", [None, 2]), inv(1, "read", None), ok(1, "read", 2)],
        [inv(0, "write", 1), ok(0, "write", 1), inv(0, "write", 2), ok(0, "write", 2),
         inv(1, "read", None), ok(1, "read", 1)],
        [inv(0, "read", None), ok(0, "read", None)],
        [inv(0, "write", -7), ok(0, "write", -7), inv(1, "read", None), ok(1, "read", -7)],
    ]
    for i, h in enumerate(cases):
        cols = H.encode(h, keyed=False)
        for init in (None, 0):
            g = ctx.check_cas(cols, init=init)
            c = oracle.check_cas(cols, init=A.NIL if init is None else init)
            assert tuple(g) == tuple(c), (i, init, g, c)


def test_keys_without_client_ops_and_unkeyed(ctx):
    """A key seen only on a nemesis entry still gets a (valid, empty) result;
    a client op whose value is not a tuple belongs to EVERY key
    (independent.clj:234-245) -- the device path reports EUNSUPPORTED and the
    host falls back to per-key calls."""
    from jepsen_amd import checker, independent, model
    t = independent.tuple_
    h = [{"process": 0, "type": "invoke", "f": "write", "value": t("a", 1)},
         {"process": 0, "type": "ok", "f": "write", "value": t("a", 1)},
         {"process": "nemesis", "type": "info", "f": "start", "value": t("b", None)}]
    r = checker.check(independent.checker(checker.linearizable({"model": model.cas_register()})),
                      {}, h, {})
    assert r["valid?"] is True and set(r["results"]) == {"a", "b"}
    h2 = h + [{"process": 1, "type": "invoke", "f": "read", "value": None},
              {"process": 1, "type": "ok", "f": "read", "value": 1}]
    r = checker.check(independent.checker(checker.linearizable({"model": model.cas_register()})),
                      {}, h2, {})
    # key "a": write 1 then read 1 -> valid; key "b": read 1 from nil -> invalid
    assert r["results"]["a"]["valid?"] is True and r["results"]["b"]["valid?"] is False
    assert r["failures"] == ["b"]


@pytest.mark.parametrize("case", ["long_keys", "many_values", "wide_window"])
def test_search_modes(ctx, case):
    """Exercise every storage mode of the per-wave search: keys whose tables
    exceed the LDS reservation (global tables, long layer windows, deep
    stack spills), more than 255 register states (HBM-only memo), windows
    wider than 40 (HBM-only memo)."""
    kw = dict(n_keys=60, ops_per_key=1500, p_invalid=0.2, p_info=0.03, seed=4242)
    if case == "many_values":
        kw.update(n_keys=200, ops_per_key=200, n_values=600)
    if case == "wide_window":
        kw.update(n_keys=40, ops_per_key=300, threads_per_key=44, readers=10, groups=44,
                  process_limit=10 ** 6, p_info=0.0)
    cols, _ = synth.cas_register(**kw)
    c, _ = oracle.check_cas_independent(cols, budget=20000, threads=8)
    g, _ = ctx.check_cas_independent(cols, budget=20000)
    _same(g, c)


def test_mutex_and_register_models(ctx):
    """knossos.model/mutex and register through the device search (the
    cas-register over {0 free, 1 held} / read-write only), single history and
    independent keys, against the oracle on the translated history."""
    from jepsen_amd import checker as CK
    from jepsen_amd import independent as IND
    from jepsen_amd import model as M
    acq = lambda p, t, v=None: {"process": p, "type": t, "f": "acquire", "value": v}
    rel = lambda p, t, v=None: {"process": p, "type": t, "f": "release", "value": v}
    good = [acq(0, "invoke"), acq(0, "ok"), rel(0, "invoke"), rel(0, "ok"), acq(1, "invoke"), acq(1, "ok")]
    bad = [acq(0, "invoke"), acq(0, "ok"), acq(1, "invoke"), acq(1, "ok")]
    lin = CK.linearizable({"model": M.mutex()})
    assert lin.check(None, good, {})["valid?"] is True
    assert lin.check(None, bad, {})["valid?"] is False
    # independent: key "a" good, key "b" bad
    h = []
    for k, hist in (("a", good), ("b", bad)):
        for op in hist:
            h.append(dict(op, process=op["process"] + (10 if k == "b" else 0), value=H.tuple_(k, None)))
    r = IND.IndependentChecker(lin).check(None, h, {})
    assert r["results"]["a"]["valid?"] is True and r["results"]["b"]["valid?"] is False
    assert r["failures"] == ["b"] and r["valid?"] is False
    # random mutex histories: device == oracle on the translated encoding
    cols_ops = []
    import random
    rng = random.Random(3)
    for key in range(200):
        busy = {}
        for _ in range(40):
            p = rng.randrange(4) + 10 * key
            if p in busy:
                cols_ops.append({"process": p, "type": rng.choice(["ok", "ok", "fail"]), "f": busy.pop(p),
                                 "value": H.tuple_(key, None)})
            else:
                f = rng.choice(["acquire", "release"])
                busy[p] = f
                cols_ops.append({"process": p, "type": "invoke", "f": f, "value": H.tuple_(key, None)})
    cols = H.encode(M.to_device_ops(M.mutex(), cols_ops), keyed=True)
    g, _ = ctx.check_cas_independent(cols, init=0)
    c, _ = oracle.check_cas_independent(cols, init=0)
    _same(g, c)
    # register: read/write only; a :cas op has no clause -> :unknown via check-safe
    reg = CK.linearizable({"model": M.register(0)})
    w = [{"process": 0, "type": "invoke", "f": "write", "value": 1},
         {"process": 0, "type": "ok", "f": "write", "value": 1},
         {"process": 1, "type": "invoke", "f": "read", "value": None},
         {"process": 1, "type": "ok", "f": "read", "value": 1}]
    assert reg.check(None, w, {})["valid?"] is True
    r = CK.check_safe(reg, None, w + [{"process": 2, "type": "invoke", "f": "cas", "value": [1, 2]}], {})
    assert r["valid?"] == CK.UNKNOWN


@pytest.mark.parametrize("seed,init", [(21, None), (22, 0), (23, None)])
def test_bfs_exact_counts(ctx, seed, init):
    """The BFS alone (JH_LIN_BFS_ONLY: no sequential search in the race) settles
    every deferred key -- invalid ones by their whole reachable set, valid ones
    by liveness + first-live-child path + closure of the dead children
    (bfs_wgl_count) -- with WGL's exact cache size, equal to the oracle's."""
    cols, _ = synth.cas_register(n_keys=150, ops_per_key=300, threads_per_key=12, readers=6, groups=10,
                                 p_info=0.0, p_invalid=0.05, nemesis_every=0, init_nil=init is None, seed=seed)
    v, s = ctx.check_cas_independent(cols, init=init, flags=A.LIN_BFS_ONLY)
    ov, _ = oracle.check_cas_independent(cols, init=A.NIL if init is None else init, threads=8)
    deferred = ov["explored"] > 4096
    assert deferred.sum() >= 5 and (ov["valid"][deferred] == A.VALID).sum() >= 3
    _same(v, ov)


def test_memo_generation_wrap():
    """the memo tables are generation-tagged and cleared only
    when the 24-bit generation range wraps. A first call leaves entries tagged
    with generations from 0; the second call is forced to wrap (JH_LIN_GEN_JUMP),
    restarts at generation 0 and must clear every table (phase 1, phase 2's
    sequential search, the helpers, phase 3) before its searches read them,
    or the first call's configurations would look visited (C3-sized keys: the
    phase-1 searches evict to the HBM table past a few hundred inserts; a
    build without the clear fails here)."""
    from jepsen_amd import _native
    ctx = _native.Context(0)
    cols, _ = synth.cas_register(n_keys=400, ops_per_key=500, p_invalid=0.02, p_info=0.02, seed=97)
    c, _ = oracle.check_cas_independent(cols, threads=8)
    g1, _ = ctx.check_cas_independent(cols)
    _same(g1, c)
    g2, _ = ctx.check_cas_independent(cols, flags=A.LIN_GEN_JUMP)
    _same(g2, c)
    ctx.close()


@pytest.mark.parametrize("seed,kw", [
    (41, dict(n_keys=300, ops_per_key=200, p_invalid=0.2, p_info=0.05)),
    (42, dict(n_keys=200, ops_per_key=300, threads_per_key=12, readers=6, p_invalid=0.1, p_info=0.02)),
    (43, dict(n_keys=40, ops_per_key=260, threads_per_key=60, readers=20, groups=60, process_limit=10 ** 6,
              p_info=0.08, p_invalid=0.2)),
])
def test_linear_algorithm(ctx, seed, kw):
    """{:algorithm :linear} (checker.clj:141-145): JIT linearization -- the
    reachable configuration set, layer by layer -- decides every key the
    device's reachable-set engine holds (:analyzer :linear, explored = the
    configurations it visited); WGL decides the rest (wide windows, sets
    past the budget: :analyzer :wgl). Every field equals the oracle's
    restatement, and :valid? equals the WGL analysis' on every key."""
    cols, _ = synth.cas_register(seed=seed, **kw)
    budget = 30000
    g, gs = ctx.check_cas_independent(cols, budget=budget, algorithm="linear")
    c, _ = oracle.check_cas_independent(cols, budget=budget, threads=16, algorithm="linear")
    _same(g, c)
    w, _ = ctx.check_cas_independent(cols, budget=budget)
    decided = (g["valid"] != A.UNKNOWN) & (w["valid"] != A.UNKNOWN)
    assert (g["valid"][decided] == w["valid"][decided]).all()
    assert (w["analyzer"] == A.ANALYZER_WGL).all()
    if seed == 43:
        # windows of up to 60 members: every key past the reachable-set
        # engine's 32, so WGL decides each one (knossos' competition fallback)
        assert (g["analyzer"] == A.ANALYZER_WGL).all()
    else:
        assert (g["analyzer"] == A.ANALYZER_LINEAR).sum() > 0


def test_linear_algorithm_host_mirror(ctx):
    """checker.Linearizable({:algorithm "linear"}) reports :analyzer :linear on
    the reference's perf_test history (valid, perf_test.clj:13-137) and keeps
    :valid? true; competition reports :wgl."""
    from jepsen_amd import checker, model
    d = json.load(open(os.path.join(GOLD, "perf_test.json")))
    r = checker.Linearizable({"model": model.CASRegister(0), "algorithm": "linear"}).check(None, d["history"], {})
    assert r["valid?"] is True and r["analyzer"] == "linear"
    r = checker.Linearizable({"model": model.CASRegister(0)}).check(None, d["history"], {})
    assert r["valid?"] is True and r["analyzer"] == "wgl"


@pytest.mark.parametrize("seed,init,kw", [
    (51, None, dict(n_keys=200, ops_per_key=200, p_invalid=0.3, p_info=0.05)),
    (52, 0, dict(n_keys=120, ops_per_key=300, threads_per_key=12, readers=6, p_invalid=0.3, p_info=0.02)),
])
def test_frontier_configs(ctx, seed, init, kw):
    """knossos' :configs (checker.clj:146-158, row f1): jh_lin_configs
    returns an invalid key's frontier -- the configurations of the last layer
    the analysis reaches -- and (ABI 6) a valid key's final configurations, in
    the canonical order, the first 10 -- register value, linearized and
    pending ops, :last-op row -- equal to the oracle's restatement key by key."""
    cols, _ = synth.cas_register(seed=seed, init_nil=init is None, **kw)
    iv = A.NIL if init is None else init
    c, _ = oracle.check_cas_independent(cols, init=iv, threads=16)
    bad = np.nonzero(c["valid"] == A.INVALID)[0]
    good = np.nonzero(c["valid"] == A.VALID)[0][:5]
    assert len(bad) >= 3
    keys = np.concatenate([bad, good])
    g = ctx.lin_configs(cols, keys, init=init)
    o = oracle.lin_configs(cols, keys, init=iv)
    assert g == o
    assert sum(1 for k in bad if g[int(k)]) >= 3
    assert sum(1 for k in good if g[int(k)]) >= 3
    assert all(all(c[3] >= 0 for c in g[int(k)]) for k in good if g[int(k)])


def test_linear_tutorial_map(ctx):
    """The reference's printed :linear analysis (doc/tutorial/04-checker.md:
    126-138), whole map, from the device path: {:valid? true :configs
    ({:model {:value 1} :last-op {... :type :ok ... :index 151} :pending []})
    :analyzer :linear :final-paths ()}; under WGL (the default competition)
    the same history gives :configs () and :final-paths ()."""
    from jepsen_amd import checker, model
    d = json.load(open(os.path.join(GOLD, "linear_tutorial.json")))
    r = checker.linearizable({"model": model.cas_register(), "algorithm": "linear"}).check({}, d["history"], {})
    assert r == d["expected"]
    r = checker.linearizable({"model": model.cas_register()}).check({}, d["history"], {})
    assert r == {"valid?": True, "configs": [], "analyzer": "wgl", "final-paths": []}


@pytest.mark.parametrize("seed", [61, 62])
def test_final_configs_crashed(ctx, seed):
    """Final configurations of valid keys with crashed ops (ABI 6): which
    crashed ops stand linearized, the value, and the :ok op each terminal edge
    linearized last, equal to the oracle's key by key; through the
    independent checker under :linear every valid key's map carries them."""
    from jepsen_amd import checker, independent, model
    cols, _ = synth.cas_register(n_keys=150, ops_per_key=120, threads_per_key=6, readers=2, p_info=0.15,
                                 p_invalid=0.1, seed=seed)
    c, _ = oracle.check_cas_independent(cols, init=A.NIL, algorithm="linear", threads=16)
    good = np.nonzero((c["valid"] == A.VALID) & (c["analyzer"] == A.ANALYZER_LINEAR))[0]
    g = ctx.lin_configs(cols, good)
    o = oracle.lin_configs(cols, good, init=A.NIL)
    assert g == o
    assert sum(1 for k in good if g[int(k)] and any(c_[1] or c_[2] for c_ in g[int(k)])) >= 5
    hist = [H.decode_op(cols, i) for i in range(cols.n)]
    r = independent.checker(checker.linearizable({"model": model.cas_register(), "algorithm": "linear"}))
    res = r.check({}, hist, {})["results"]
    for k in good[:40]:
        m = res[cols.keys[int(k)]]
        assert m["valid?"] is True and m["analyzer"] == "linear" and m["final-paths"] == []
        assert len(m["configs"]) == len(g[int(k)])
        for cfg, (v, lin, pend, last) in zip(m["configs"], g[int(k)]):
            assert cfg["model"] == {"value": None if v == A.NIL else v}
            assert cfg["last-op"]["index"] == last and cfg["last-op"]["type"] == "ok"
            assert [p_["index"] for p_ in cfg["pending"]] == pend


def test_frontier_configs_host_map(ctx):
    """checker.Linearizable on the reference's perf_test history with a nil
    initial value (invalid: the first read of 0 cannot be linearized) carries
    :configs and :final-paths, at most 10 of each, every pending op a map of
    the history."""
    from jepsen_amd import checker, model
    d = json.load(open(os.path.join(GOLD, "perf_test.json")))
    r = checker.Linearizable({"model": model.CASRegister(None)}).check(None, d["history"], {})
    assert r["valid?"] is False and 0 < len(r["configs"]) <= 10 and len(r["final-paths"]) == len(r["configs"])
    for cfg in r["configs"]:
        assert set(cfg) == {"model", "last-op", "pending"}
        assert all(op["type"] == "invoke" for op in cfg["pending"])
        # as knossos prints it (doc/tutorial/04-checker.md:128-135): the :ok
        # completion of the last op linearized, with its own :index
        if cfg["last-op"] is not None:
            i = cfg["last-op"]["index"]
            assert cfg["last-op"]["type"] == "ok" and dict(d["history"][i], index=i) == cfg["last-op"]
    for p in r["final-paths"]:
        assert p[-1]["op"] == r["op"] and "inconsistent" in p[-1]["model"]


@pytest.mark.parametrize("seed", [3, 3 + 7919 * 3])
def test_streamed_equals_round3_schedule(ctx, seed):
    """The streaming heavy-key pass (JH_LIN_STREAM: consumers start while
    phase 1 still defers keys) and the default schedule (after phase 1)
    decide every key identically, and both equal the oracle; a 2 000-key slice
    of the C3 workload (rank 0 / rank 3 seeds) has keys in every engine."""
    cols, _ = synth.cas_register(n_keys=2000, ops_per_key=500, threads_per_key=10, readers=5, n_values=5,
                                 process_limit=20, groups=10, p_info=0.02, p_invalid=0.01, nemesis_every=10000,
                                 seed=seed)
    g, gs = ctx.check_cas_independent(cols, flags=A.LIN_STREAM)
    # the default schedule without the hand-over (round 5 hands long searches
    # over once phase 1's queue is empty; the streaming pass keeps them)
    l, ls = ctx.check_cas_independent(cols, flags=A.LIN_NO_HANDOVER)
    assert gs.streamed == 1 and ls.streamed == 0
    assert gs.n_deferred == ls.n_deferred > 0
    _same(g, l)
    c, _ = oracle.check_cas_independent(cols, threads=8)
    _same(g, c)


@pytest.mark.parametrize("quick", [300, 2000, 30000])
def test_phase1_quick_budgets(ctx, quick):
    """Phase 1 at quick budgets from one LDS eviction's worth to past the
    heavy keys' size (keys past it deferred): every field equal to the
    oracle."""
    cols, _ = synth.cas_register(n_keys=300, ops_per_key=400, threads_per_key=10, readers=5, groups=10,
                                 p_info=0.05, p_invalid=0.1, seed=4242)
    g, gs = ctx.check_cas_independent(cols, quick_budget=quick)
    c, _ = oracle.check_cas_independent(cols, threads=8)
    _same(g, c)


def _wide_failure_history(widths):
    """One key per width P: a read of a never-written value fails at the
    sixth row (three writes concurrent with it), after which P crashed
    writes stay open to the end -- the key's widest window is P + 1 members,
    so the whole key runs in the 33-64 (P < 64) or 65-256-member engine
    while its frontier is small and exact."""
    h = []
    for k, p in enumerate(widths):
        t = lambda v: H.tuple_(k, v)  # noqa: E731
        h += [H.invoke_op(0, "write", t(1)), H.ok_op(0, "write", t(1)),
              H.invoke_op(1, "write", t(2)), H.invoke_op(2, "write", t(3)), H.invoke_op(3, "read", t(None)),
              H.ok_op(3, "read", t(4)), H.ok_op(1, "write", t(2)), H.ok_op(2, "write", t(3))]
        h += [H.invoke_op(100 + i, "write", t(1 + i % 3)) for i in range(p)]
        h += [H.invoke_op(4, "read", t(None)), H.ok_op(4, "read", t(1))]
        h += [H.info_op(100 + i, "write", t(1 + i % 3)) for i in range(p)]
    return H.encode(h)


def test_frontier_configs_wide_windows(ctx):
    """:configs beyond the reachable-set engine (round 4, row f1): keys whose
    windows exceed 32 members take their frontier from the WIDE / 65-256
    member search's table; the configurations equal the oracle's
    (orc_linear's frontier, any window) key by key. Two histories: synthetic
    keys of 40 threads (windows 36-40, invalid deep in the history) and
    hand-made keys whose windows reach 41, 71, 131 and 251 members."""
    cols, _ = synth.cas_register(n_keys=48, ops_per_key=40, threads_per_key=40, readers=20, n_values=5,
                                 process_limit=320, groups=10, init_nil=True, p_info=0.3, p_invalid=0.6,
                                 nemesis_every=10000, seed=556)
    budget = 1 << 18
    c, _ = oracle.check_cas_independent(cols, budget=budget, threads=16)
    bad = np.nonzero(c["valid"] == A.INVALID)[0]
    assert len(bad) >= 3
    g = ctx.lin_configs(cols, bad, budget=budget)
    o = oracle.lin_configs(cols, bad, budget=budget)
    assert g == o
    assert all(g[int(k)] for k in bad)

    cols = _wide_failure_history([40, 70, 130, 250])
    keys = np.arange(4)
    c, _ = oracle.check_cas_independent(cols, budget=1 << 16, threads=4)
    assert (c["valid"] == A.INVALID).all()
    g = ctx.lin_configs(cols, keys, budget=1 << 16)
    o = oracle.lin_configs(cols, keys, budget=1 << 16)
    assert g == o
    assert all(len(g[k]) == 5 for k in range(4))


@pytest.mark.parametrize("case", ["bfs_only", "c3_budget22"])
def test_uncounted_early_emit(ctx, case):
    """The checkers' own path: without
    JH_LIN_EXACT_COUNT, a valid key the reachable-set engine settles with at
    most `budget` configurations reachable is emitted at once with explored
    = JH_EXPLORED_UNCOUNTED (jh_lin.hip, the early emit after the forward
    pass). Forced two ways -- the BFS alone (JH_LIN_BFS_ONLY) on keys whose
    reachable sets fit it, and the benched C3 configuration itself (seed 3,
    budget 2^22) -- every key's verdict, cause and failing row equal the
    oracle's, every uncounted key is valid in the oracle, and every counted
    key's explored equals WGL's count."""
    if case == "bfs_only":
        cols, _ = synth.cas_register(n_keys=150, ops_per_key=300, threads_per_key=12, readers=6, groups=10,
                                     p_info=0.0, p_invalid=0.05, nemesis_every=0, init_nil=True, seed=21)
        g, _ = ctx.check_cas_independent(cols, flags=A.LIN_BFS_ONLY, exact_count=False)
        c, _ = oracle.check_cas_independent(cols, threads=8)
    else:
        cols, _ = synth.cas_register(seed=3)
        g, _ = ctx.check_cas_independent(cols, budget=1 << 22, exact_count=False)
        c, _ = oracle.check_cas_independent(cols, budget=1 << 22, threads=16)
    unc = g["explored"] == A.EXPLORED_UNCOUNTED
    # the BFS alone settles many valid keys (forced); on C3 the race leaves it
    # the few it wins, zero or a handful by timing (the helpers and the spec
    # board often settle them first), so only the fields are checked there
    if case == "bfs_only":
        assert unc.sum() >= 5, unc.sum()
    assert (c["valid"][unc] == A.VALID).all()
    for f in ("valid", "cause", "fail_entry"):
        bad = np.nonzero(g[f] != c[f])[0]
        assert len(bad) == 0, (f, bad[:10])
    bad = np.nonzero((g["explored"] != c["explored"]) & ~unc)[0]
    assert len(bad) == 0, ("explored", bad[:10], g[bad[:5]], c[bad[:5]])


@pytest.mark.parametrize("seed", [14, 16, 18])
def test_configs_list_dropped_reads_device(ctx, seed):
    """Round 6: jh_lin_configs lists the reads the search
    drops -- crashed reads, :ok reads of nil -- in :pending as knossos holds
    them, and moves :last-op to a read of nil that completes later (the
    oracle's restatement is pinned on the strict just-in-time linearization,
    tests/test_oracle_crosscheck.py::test_configs_list_dropped_reads): the
    device equals the oracle on every invalid key's frontier and every valid
    :linear key's final configurations, and some list such reads."""
    cols, _ = synth.cas_register(n_keys=300, ops_per_key=40, threads_per_key=4, readers=2, n_values=3,
                                 process_limit=10 ** 6, p_info=0.15, p_invalid=0.3, nemesis_every=10 ** 9,
                                 init_nil=True, seed=seed)
    c, _ = oracle.check_cas_independent(cols, init=A.NIL, algorithm="linear", threads=16)
    keys = np.nonzero((c["valid"] == A.INVALID) | ((c["valid"] == A.VALID) & (c["analyzer"] == A.ANALYZER_LINEAR)))[0]
    g = ctx.lin_configs(cols, keys)
    o = oracle.lin_configs(cols, keys, init=A.NIL)
    assert g == o
    from jepsen_amd.checker import _next_same_process
    nxt = _next_same_process(cols)
    noop = set()
    for r in np.nonzero((cols.f == A.F_READ) & (cols.type == A.TYPE_INVOKE))[0].tolist():
        q = int(nxt[r])
        if q < 0 or cols.type[q] == A.TYPE_INFO or (cols.type[q] == A.TYPE_OK and cols.value[q] == A.NIL):
            noop.add(r)
    assert sum(1 for k in keys if g[int(k)] and any(set(p) & noop for _, _, p, _ in g[int(k)])) >= 5


@pytest.mark.parametrize("rank,keys", [(0, [1086, 8979, 4457, 8190]), (4, [1631, 4356])])
def test_spec_dead_subtrees(ctx, rank, keys):
    """Round 6: idle late helpers enumerate dead-subtree
    candidates the key's exact search posts (SpecSlot) and the search merges
    the dead ones: on the C3 keys that end the step (rank 0's 1086 / 8979 /
    4457 / 8190, rank 4's 1631), one big dead subtree each
    (tools/shape/wgl_shape.py), every field -- WGL's count included -- equals
    the oracle's, with merges made, at the full budget and at one the merged
    searches run into; the same without the board (JH_LIN_NO_SPEC)."""
    from jepsen_amd import shard
    from bench import WORKLOADS
    wl = WORKLOADS["c3"]
    cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"] + 7919 * rank, **wl["gen"])
    own = np.ones(cols.n_keys, np.int64)
    own[keys] = 0
    sub, mine, _ = shard.shard_history(cols, own, 0)
    merged = 0
    for budget in (1 << 22, 20000):
        c, _ = oracle.check_cas_independent(sub, budget=budget, threads=8)
        g, s = ctx.check_cas_independent(sub, budget=budget, flags=A.LIN_HELPERS_NOW)
        _same(g, c)
        merged += s.spec_merges
        stats = (budget, s.spec_jobs, s.spec_dead, s.spec_merges, s.spec_nodes)
        print("spec jobs / dead / merges / nodes at budget", stats)
        assert s.spec_nodes >= 0 and s.spec_dead >= s.spec_merges, stats
        g2, s2 = ctx.check_cas_independent(sub, budget=budget, flags=A.LIN_HELPERS_NOW | A.LIN_NO_SPEC)
        _same(g2, c)
        assert s2.spec_jobs == 0 and s2.spec_merges == 0
        # the scheduling variants: helpers serving the board first, helpers
        # picking the keys stuck longest (JH_LIN_SPEC_FIRST, JH_LIN_HELP_STALL)
        for fl in (A.LIN_SPEC_FIRST, A.LIN_HELP_STALL | A.LIN_SPEC_FIRST):
            g3, s3 = ctx.check_cas_independent(sub, budget=budget, flags=fl, helper_late_us=100)
            _same(g3, c)
    assert merged > 0


@pytest.mark.parametrize("rank,keys", [(0, [1086, 8979, 4457, 8190, 932, 3101]), (4, [1631, 4356])])
def test_takeover(ctx, rank, keys):
    """Round 6, the takeover: a late helper that takes a key phase 2's
    sequential search is running asks that search for its state (it saves its
    record at its next check and leaves the key) and continues it in dfs_acc
    instead of restarting it. On the C3 keys that end the step, with the
    helpers taking keys after 1 ms (so the sequential searches are well under
    way), every field -- WGL's count included -- equals the oracle's at the
    full budget and at one the searches run into, with takeovers made; the
    same with JH_LIN_NO_TAKEOVER and none made."""
    from jepsen_amd import shard
    from bench import WORKLOADS
    wl = WORKLOADS["c3"]
    cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"] + 7919 * rank, **wl["gen"])
    own = np.ones(cols.n_keys, np.int64)
    own[keys] = 0
    sub, mine, _ = shard.shard_history(cols, own, 0)
    took = 0
    for budget in (1 << 22, 20000):
        c, _ = oracle.check_cas_independent(sub, budget=budget, threads=8)
        for late in (1000, 3000):
            g, s = ctx.check_cas_independent(sub, budget=budget, flags=A.LIN_TAKEOVER, helper_late_us=late)
            _same(g, c)
            took += s.takeovers
            print("takeovers at budget", budget, "late", late, s.takeovers, "spec merges", s.spec_merges)
        g2, s2 = ctx.check_cas_independent(sub, budget=budget, helper_late_us=1000)      # the default: off
        _same(g2, c)
        assert s2.takeovers == 0
    assert took > 0
