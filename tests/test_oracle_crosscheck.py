"""Independent CPU formulations of linearizability must agree (no GPU).

canonical WGL (what libjh.so implements) == knossos-style linked-list WGL
(verdict AND cache size) == brute-force linearization search (verdict), and
for invalid keys the WGL cache equals the full reachable configuration set."""
import ctypes as C

import numpy as np
import pytest

from jepsen_amd import _abi as A
from jepsen_amd import history as H
from jepsen_amd import synth
from oracle import oracle


def _sub(cols, k):
    sel = np.nonzero((cols.key == k) | (cols.key < 0))[0]
    return H.Columns(n=len(sel), process=cols.process[sel].copy(), type=cols.type[sel].copy(),
                     f=cols.f[sel].copy(), key=np.full(len(sel), -1, np.int64),
                     value=cols.value[sel].copy(), value2=cols.value2[sel].copy(), n_keys=0,
                     aux=cols.aux)


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_three_formulations_agree_tiny(built, seed):
    cols, _ = synth.cas_register(n_keys=600, ops_per_key=7, threads_per_key=4, readers=1, groups=5,
                                 p_info=0.15, p_invalid=0.3, nemesis_every=7, seed=seed)
    counts = {A.VALID: 0, A.INVALID: 0}
    for k in range(cols.n_keys):
        r = oracle.key_selftest(_sub(cols, k))
        assert r["status"] == 0
        assert r["canonical"] == r["list"], r
        assert r["canonical_explored"] == r["list_explored"], r
        assert r["bruteforce"] in (r["canonical"], -1), r
        counts[r["canonical"]] += 1
    assert counts[A.INVALID] > 10 and counts[A.VALID] > 10


def test_init_value_variants(built):
    cols, _ = synth.cas_register(n_keys=300, ops_per_key=8, threads_per_key=3, readers=1,
                                 groups=3, p_info=0.1, p_invalid=0.2, seed=21, init_nil=False)
    for k in range(cols.n_keys):
        for init in (0, A.NIL, 3):
            r = oracle.key_selftest(_sub(cols, k), init=init)
            assert r["canonical"] == r["list"] and r["canonical_explored"] == r["list_explored"]
            assert r["bruteforce"] in (r["canonical"], -1)


def test_invalid_keys_explore_whole_reachable_set(built):
    cols, _ = synth.cas_register(n_keys=150, ops_per_key=60, threads_per_key=6, readers=2,
                                 groups=3, p_info=0.05, p_invalid=0.3, seed=31)
    L = oracle.lib()
    L.orc_key_stats.argtypes = [C.POINTER(A.JhHistory), C.c_int64, C.c_int64, C.c_int64,
                                C.c_int64, C.c_int64, C.POINTER(C.c_int64)]
    h = cols.as_jh()
    res = np.zeros(6 * cols.n_keys, np.int64)
    L.orc_key_stats(C.byref(h), A.NIL, A.DEFAULT_BUDGET, 1 << 22, 0, cols.n_keys, A.ptr64(res))
    r = res.reshape(-1, 6)
    assert (r[:, 0] == r[:, 2]).all()                 # same verdict
    inv = r[:, 0] == A.INVALID
    assert inv.sum() > 5
    assert (r[inv, 1] == r[inv, 3]).all()             # explored == |reachable|


def test_faithful_split_equals_bucketed(built):
    """independent.clj:234-245's O(K*N) subhistory == the O(N) bucketed split."""
    cols, _ = synth.cas_register(n_keys=120, ops_per_key=50, seed=41, nemesis_every=30)
    a, sa = oracle.check_cas_independent(cols, mode=0)
    b, sb = oracle.check_cas_independent(cols, mode=1, threads=4)
    assert (a == b).all()
    assert sa.valid == sb.valid and sa.n_invalid == sb.n_invalid


def test_budget_gives_unknown(built):
    cols, _ = synth.cas_register(n_keys=50, ops_per_key=200, seed=51, p_invalid=0.2)
    v, _ = oracle.check_cas_independent(cols, budget=50)
    assert (v["valid"] == A.UNKNOWN).any()
    unk = v["valid"] == A.UNKNOWN
    assert (v["explored"][unk] == 50).all() and (v["cause"][unk] == 1).all()
    # raising the budget resolves them, and never flips a resolved verdict
    w, _ = oracle.check_cas_independent(cols)
    res = v["valid"] != A.UNKNOWN
    assert (w["valid"][res] == v["valid"][res]).all()


def test_history_completion_errors(built):
    def enc(ops):
        return H.encode(ops, keyed=False)
    inv = lambda p, f, v: {"process": p, "type": "invoke", "f": f, "value": v}
    ok = lambda p, f, v: {"process": p, "type": "ok", "f": f, "value": v}
    info = lambda p, f, v: {"process": p, "type": "info", "f": f, "value": v}
    # double invoke (knossos.history/complete throws -> :unknown)
    v = oracle.check_cas(enc([inv(0, "write", 1), inv(0, "write", 2)]))
    assert v[0] == A.UNKNOWN and A.CAUSES[v[1]] == "double-invoke"
    # an :info does not close the process: invoking again is a double invoke
    v = oracle.check_cas(enc([inv(0, "write", 1), info(0, "write", 1), inv(0, "write", 2)]))
    assert v[0] == A.UNKNOWN and A.CAUSES[v[1]] == "double-invoke"
    # completion without invocation
    v = oracle.check_cas(enc([ok(0, "write", 1)]))
    assert v[0] == A.UNKNOWN and A.CAUSES[v[1]] == "orphan-completion"
    # unknown :f on a non-failed op
    v = oracle.check_cas(enc([inv(0, "incr", 1), ok(0, "incr", 1)]))
    assert v[0] == A.UNKNOWN and A.CAUSES[v[1]] == "unsupported-f"
    # nemesis entries are ignored; empty history is valid
    v = oracle.check_cas(enc([{"process": "nemesis", "type": "info", "f": "start"}]))
    assert v[0] == A.VALID
    v = oracle.check_cas(enc([]))
    assert v[0] == A.VALID and v[3] == 0
    # a crashed write may or may not have happened
    v = oracle.check_cas(enc([inv(0, "write", 3), info(0, "write", 3), inv(1, "read", None),
                              ok(1, "read", 3), inv(2, "read", None), ok(2, "read", 3)]))
    assert v[0] == A.VALID
    v = oracle.check_cas(enc([inv(0, "write", 3), info(0, "write", 3), inv(1, "read", None),
                              ok(1, "read", None)]))
    assert v[0] == A.VALID
    # a stale read after a completed write is not
    v = oracle.check_cas(enc([inv(0, "write", 1), ok(0, "write", 1), inv(0, "write", 2),
                              ok(0, "write", 2), inv(1, "read", None), ok(1, "read", 1)]))
    assert v[0] == A.INVALID and v[2] == 5


@pytest.mark.parametrize("seed", [61, 62])
def test_wide_windows_agree(built, seed):
    """Windows of 65..256 members (multi-word masks): canonical == list WGL,
    verdict and cache size, at the full budget and at a small one; wider
    than 256 is :unknown with cause window in both."""
    cols, _ = synth.cas_register(n_keys=24, ops_per_key=260, threads_per_key=120, readers=20,
                                 groups=120, process_limit=10 ** 6, p_info=0.08, p_invalid=0.2,
                                 seed=seed)
    widths, settled = [], 0
    for k in range(cols.n_keys):
        sub = _sub(cols, k)
        for budget in (3000, 40000):
            r = oracle.key_selftest(sub, budget=budget)
            widths.append(r["max_window"])
            if r["max_window"] > A.MAX_WINDOW:
                assert r["status"] == 2 and r["canonical"] == A.UNKNOWN      # cause window
                continue
            assert r["canonical"] == r["list"], r
            assert r["canonical_explored"] == r["list_explored"], r
            settled += r["canonical"] != A.UNKNOWN
    assert sum(64 < w <= A.MAX_WINDOW for w in widths) >= 8 and settled >= 2


def _jit_frontier(cols, key, init):
    """The frontier of an invalid key from the definition (knossos.linear's
    just-in-time linearization over op maps, no canonical coordinates): the
    set of (linearized ops, register value) reachable by linearizing invoked
    ops; at each :ok completion keep the configurations that linearized it.
    At the first completion no configuration can linearize, the whole closure
    is the frontier. Returns (window rows in call order, [(value, linearized
    row set)]) or None when the key is valid. :fail ops are dropped (complete
    marks them :fails?), so are :ok reads of nil (they constrain nothing:
    DESIGN §2); histories here have no :info."""
    NIL = A.NIL
    rows = [i for i in range(cols.n) if int(cols.key[i]) == key]
    open_by_proc, ops = {}, {}
    for i in rows:
        p, ty = int(cols.process[i]), int(cols.type[i])
        if ty == A.TYPE_INVOKE:
            open_by_proc[p] = i
            ops[i] = {"f": int(cols.f[i]), "v": int(cols.value[i]), "v2": int(cols.value2[i]), "ret": None}
        else:
            inv = open_by_proc.pop(p)
            if ty == A.TYPE_FAIL:
                ops[inv]["fail"] = True
            elif ty == A.TYPE_OK:
                ops[inv]["ret"] = i
                if ops[inv]["f"] == 0:               # read: the completion carries the value
                    ops[inv]["v"] = int(cols.value[i])
                    if ops[inv]["v"] == A.NIL:
                        ops[inv]["fail"] = True
    def step(s, o):
        if o["f"] == 1:
            return o["v"]
        if o["f"] == 2:
            return o["v2"] if s == o["v"] else None
        return s if (o["v"] == NIL or o["v"] == s) else None
    configs = {(frozenset(), init)}
    avail, done = set(), set()
    reach = set(configs)
    for i in rows:
        if int(cols.type[i]) == A.TYPE_INVOKE:
            if not ops[i].get("fail"):
                avail.add(i)
            continue
        if int(cols.type[i]) != A.TYPE_OK:
            continue
        inv = next((o for o in avail if ops[o]["ret"] == i), None)
        if inv is None:                              # a dropped op's completion
            continue
        seen, stack = set(configs), list(configs)
        while stack:
            L, s = stack.pop()
            for o in avail - L:
                s2 = step(s, ops[o])
                if s2 is None:
                    continue
                c = (L | {o}, s2)
                if c not in seen:
                    seen.add(c)
                    stack.append(c)
        nxt = {c for c in seen if inv in c[0]}
        reach |= seen
        if not nxt:
            window = sorted(avail - done)
            _jit_frontier.reach = len(reach)
            _jit_frontier.last = max((ops[o]["ret"] for o in done), default=-1)
            return window, sorted(seen, key=lambda c: (
                0 if c[1] == NIL else 2, c[1], sum(1 << j for j, r in enumerate(window) if r in c[0])))
        configs = nxt
        done.add(inv)
    return None


@pytest.mark.parametrize("seed", [11, 12])
def test_frontier_configs_from_definition(built, seed):
    """orc_lin_configs (the restatement jh_lin_configs is checked against on
    the GPU) equals the frontier computed from the definition by a
    just-in-time linearization over op maps: the first 10 configurations in
    the canonical order, each value, linearized window rows and pending
    window rows and the :last-op row, for every invalid key."""
    cols, _ = synth.cas_register(n_keys=60, ops_per_key=24, threads_per_key=3, readers=1, n_values=3,
                                 process_limit=10 ** 6, p_info=0.0, p_invalid=0.5, nemesis_every=10 ** 9,
                                 seed=seed)
    got = oracle.lin_configs(cols, list(range(cols.n_keys)), init=A.NIL)
    n_bad = 0
    for k in range(cols.n_keys):
        ref = _jit_frontier(cols, k, A.NIL)
        if ref is None:               # valid: its final configurations, test_final_configs_from_definition
            continue
        n_bad += 1
        window, front = ref
        want = [(v, [r for r in window if r in L], [r for r in window if r not in L]) for L, v in front][:10]
        assert [(int(v), list(map(int, lin)), list(map(int, pend))) for v, lin, pend, _ in got[k]] == want, k
        # :last-op: the completion of the last :ok op before the failing one,
        # reads of nil included (round 6: _jit_noop keeps them as ops)
        (_, _, _, last_ref), _ = _jit_noop(cols, k, A.NIL, "full")
        assert all(last == last_ref for *_, last in got[k]), k
    assert n_bad >= 5


def test_linear_analysis_from_definition(built):
    """The oracle's :linear analysis (orc_linear) against the same
    just-in-time linearization from the definition: :valid? equal to WGL's on
    every key, :analyzer :linear on every key of the reachable-set domain, and
    its explored count the reachable configurations (initial and terminal
    ones excluded) -- for invalid keys the closure sizes summed over the
    layers, which the definition recounts."""
    cols, _ = synth.cas_register(n_keys=60, ops_per_key=24, threads_per_key=3, readers=1, n_values=3,
                                 process_limit=10 ** 6, p_info=0.0, p_invalid=0.5, nemesis_every=10 ** 9,
                                 seed=13)
    lin, _ = oracle.check_cas_independent(cols, init=A.NIL, algorithm="linear")
    wgl, _ = oracle.check_cas_independent(cols, init=A.NIL)
    assert (lin["valid"] == wgl["valid"]).all()
    assert (lin["analyzer"] == A.ANALYZER_LINEAR).all()
    for k in range(cols.n_keys):
        ref = _jit_frontier(cols, k, A.NIL)
        assert (ref is None) == (int(lin["valid"][k]) == A.VALID), k
        if ref is not None:
            assert int(lin["explored"][k]) == _jit_frontier.reach - 1, k
    assert (lin["valid"] == A.INVALID).sum() >= 5


def _jit_final(cols, key, init):
    """The final configurations of a valid key from the definition: knossos'
    just-in-time linearization over op maps, strictly -- at each :ok
    completion a configuration that already linearized the op survives as it
    is; any other is expanded by linearizing pending ops, in every order,
    until the completing op is linearized, which becomes its :last-op. The
    configurations left after the history are (value, linearized ops,
    :last-op row). None when some completion leaves no configuration.
    :fail ops and :ok reads of nil are dropped (as _jit_frontier)."""
    NIL = A.NIL
    rows = [i for i in range(cols.n) if int(cols.key[i]) == key]
    open_by_proc, ops = {}, {}
    for i in rows:
        p, ty = int(cols.process[i]), int(cols.type[i])
        if ty == A.TYPE_INVOKE:
            open_by_proc[p] = i
            ops[i] = {"f": int(cols.f[i]), "v": int(cols.value[i]), "v2": int(cols.value2[i]), "ret": None}
        else:
            inv = open_by_proc.pop(p)
            if ty == A.TYPE_FAIL:
                ops[inv]["fail"] = True
            elif ty == A.TYPE_OK:
                ops[inv]["ret"] = i
                if ops[inv]["f"] == 0:
                    ops[inv]["v"] = int(cols.value[i])
                    if ops[inv]["v"] == NIL:
                        ops[inv]["fail"] = True
            elif ops[inv]["f"] == 0:                     # a crashed read never matters: dropped
                ops[inv]["fail"] = True

    def step(s, o):
        if o["f"] == 1:
            return o["v"]
        if o["f"] == 2:
            return o["v2"] if s == o["v"] else None
        return s if (o["v"] == NIL or o["v"] == s) else None
    configs = {(frozenset(), init, -1)}
    avail = set()
    for i in rows:
        if int(cols.type[i]) == A.TYPE_INVOKE:
            if not ops[i].get("fail"):
                avail.add(i)
            continue
        if int(cols.type[i]) != A.TYPE_OK:
            continue
        inv = next((o for o in avail if ops[o]["ret"] == i), None)
        if inv is None:
            continue
        new = set()
        for L, s, last in configs:
            if inv in L:
                new.add((L, s, last))
                continue
            seen, stack = {(L, s)}, [(L, s)]
            while stack:
                L2, s2 = stack.pop()
                for o in avail - L2:
                    s3 = step(s2, ops[o])
                    if s3 is None:
                        continue
                    if o == inv:
                        new.add((L2 | {o}, s3, i))
                    elif (L2 | {o}, s3) not in seen:
                        seen.add((L2 | {o}, s3))
                        stack.append((L2 | {o}, s3))
        if not new:
            return None
        configs = new
    crashed = sorted(o for o in avail if ops[o]["ret"] is None)
    return crashed, configs


def _jit_noop(cols, key, init, mode):
    """knossos' just-in-time linearization over op maps, strictly (as
    _jit_final), with the reads the search drops -- crashed reads and :ok
    reads of nil, which constrain nothing -- kept as ops (round 6, VERDICT r5
    item 1b). mode "full": they are ops like any other (knossos' own set);
    mode "lazy": such a read is linearized only when its own completion forces
    it, by itself, and never as part of another op's expansion (a crashed read
    never) -- the member of knossos' set libjh prints for each configuration
    of its search. Returns ("frontier", window rows in call order, closure
    {(L, s)}, last completion row) at the first completion no configuration
    survives, else ("final", {(L, s, last)}), plus the no-op read rows."""
    NIL = A.NIL
    rows = [i for i in range(cols.n) if int(cols.key[i]) == key]
    open_by_proc, ops = {}, {}
    for i in rows:
        p, ty = int(cols.process[i]), int(cols.type[i])
        if ty == A.TYPE_INVOKE:
            open_by_proc[p] = i
            ops[i] = {"f": int(cols.f[i]), "v": int(cols.value[i]), "v2": int(cols.value2[i]), "ret": None}
        else:
            inv = open_by_proc.pop(p, None) if ty != A.TYPE_INFO else None
            if inv is None:
                continue
            if ty == A.TYPE_FAIL:
                ops[inv]["fail"] = True
            elif ty == A.TYPE_OK:
                ops[inv]["ret"] = i
                if ops[inv]["f"] == 0 and ops[inv]["v"] == NIL:
                    ops[inv]["v"] = int(cols.value[i])
    noop = {o for o, d in ops.items() if not d.get("fail") and d["f"] == 0 and (d["ret"] is None or d["v"] == NIL)}

    def step(s, o):
        if o["f"] == 1:
            return o["v"]
        if o["f"] == 2:
            return o["v2"] if s == o["v"] else None
        return s if (o["v"] == NIL or o["v"] == s) else None
    configs = {(frozenset(), init, -1)}
    avail, done = set(), set()
    for i in rows:
        if int(cols.type[i]) == A.TYPE_INVOKE:
            if not ops[i].get("fail"):
                avail.add(i)
            continue
        if int(cols.type[i]) != A.TYPE_OK:
            continue
        inv = next((o for o in avail if ops[o]["ret"] == i), None)
        if inv is None:
            continue
        cand = avail if mode == "full" else avail - noop
        new, closure = set(), set()
        for L, s, last in configs:
            if inv in L:
                new.add((L, s, last))
                continue
            if mode == "lazy" and inv in noop:
                new.add((L | {inv}, s, i))
                continue
            seen, stack = {(L, s)}, [(L, s)]
            while stack:
                L2, s2 = stack.pop()
                for o in cand - L2:
                    s3 = step(s2, ops[o])
                    if s3 is None:
                        continue
                    if o == inv:
                        new.add((L2 | {o}, s3, i))
                    elif (L2 | {o}, s3) not in seen:
                        seen.add((L2 | {o}, s3))
                        stack.append((L2 | {o}, s3))
            closure |= seen
        if not new:
            last = max((ops[o]["ret"] for o in done), default=-1)
            return ("frontier", sorted(avail - done), closure | {(L, s) for L, s, _ in configs}, last), noop
        configs = new
        done.add(inv)
    return ("final", configs), noop


@pytest.mark.parametrize("seed", [14, 15, 16, 17, 18])
def test_configs_list_dropped_reads(built, seed):
    """Round 6: :pending lists the reads the search
    drops, as knossos' analysis holds them (checker.clj:156-158). Checked
    against the strict just-in-time linearization with those reads kept as
    ops, on histories with crashed reads and :ok reads of nil:
      - an invalid key's frontier is exactly knossos' closure at the failing
        completion restricted to the configurations that linearized none of
        the reads still open there, first 10 in the canonical order, every
        open read pending, :last-op the last completion before the failure;
      - a valid key's final configurations are exactly the set in which such
        a read is linearized only when its own completion forces it, and
        every one of them is in knossos' own (full) set -- which crashed ops
        stand linearized, the value and :last-op, the :ok op (a read of nil
        included) each configuration linearized last (round 5's
        test_final_configs_from_definition, with the dropped reads kept)."""
    cols, _ = synth.cas_register(n_keys=60, ops_per_key=24, threads_per_key=3, readers=2, n_values=3,
                                 process_limit=10 ** 6, p_info=0.15, p_invalid=0.3, nemesis_every=10 ** 9,
                                 init_nil=True, seed=seed)
    lin, _ = oracle.check_cas_independent(cols, init=A.NIL, algorithm="linear")
    got = oracle.lin_configs(cols, list(range(cols.n_keys)), init=A.NIL)
    n_front = n_final = n_noop_pending = n_crashed = 0
    for k in range(cols.n_keys):
        (kind, *rest), noop = _jit_noop(cols, k, A.NIL, "full")
        if kind == "frontier":
            window, closure, last = rest
            assert int(lin["valid"][k]) == A.INVALID, k
            opened = set(window) & noop
            red = [r for r in window if r not in noop]
            keep = [(L, s) for L, s in closure if not (L & opened)]
            keep.sort(key=lambda c: (0 if c[1] == A.NIL else 2, c[1], sum(1 << j for j, r in enumerate(red) if r in c[0])))
            want = [(s, [r for r in window if r in L], [r for r in window if r not in L], last) for L, s in keep][:10]
            assert got[k] == want, k
            n_front += 1
            n_noop_pending += bool(opened)
            continue
        full = rest[0]
        if int(lin["valid"][k]) != A.VALID or got[k] is None:
            continue
        (_, lazy), _ = _jit_noop(cols, k, A.NIL, "lazy")
        assert lazy <= full, k
        rows = sorted(set().union(*(L for L, _, _ in lazy)) | {o for o in noop if int(cols.type[o]) == A.TYPE_INVOKE})
        crashed = sorted(r for r in _jit_final(cols, k, A.NIL)[0])
        cr_noop = sorted(o for o in noop if all(int(cols.process[j]) != int(cols.process[o]) or
                                                int(cols.type[j]) != A.TYPE_OK for j in range(o + 1, cols.n)
                                                if int(cols.key[j]) == k))
        order = sorted(lazy, key=lambda c: (0 if c[1] == A.NIL else 2, c[1],
                                            sum(1 << j for j, r in enumerate(crashed) if r in c[0]), c[2]))
        want = [(s, [r for r in crashed if r in L], sorted([r for r in crashed if r not in L] + cr_noop), last)
                for L, s, last in order][:10]
        assert got[k] == want, (k, rows)
        n_final += 1
        n_noop_pending += bool(cr_noop)
        n_crashed += any(c[1] or set(c[2]) - set(cr_noop) for c in want)
    assert n_front >= 5 and n_final >= 5 and n_noop_pending >= 3 and n_crashed >= 3
