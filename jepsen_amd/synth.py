"""Seeded synthetic histories from libjhgen.so.

Workload generator for bench.py and the tests: the histories are shaped like
the reference workloads (see csrc/gen.cpp header) and are returned as
`history.Columns` (host numpy int64 columns in the include/jh.h layout).
"""
import ctypes as C
import os

import numpy as np

from .history import Columns

JH_NIL = -(1 << 63)

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


class _CasParams(C.Structure):
    _fields_ = [("n_keys", C.c_int64), ("ops_per_key", C.c_int64),
                ("threads_per_key", C.c_int32), ("readers", C.c_int32),
                ("n_values", C.c_int32), ("process_limit", C.c_int32),
                ("groups", C.c_int32), ("init_nil", C.c_int32),
                ("p_info", C.c_double), ("p_invalid", C.c_double),
                ("nemesis_every", C.c_int64), ("seed", C.c_uint64),
                ("keyed", C.c_int32), ("pad", C.c_int32)]


class _CounterParams(C.Structure):
    _fields_ = [("n_ops", C.c_int64), ("n_procs", C.c_int32), ("read_every", C.c_int32),
                ("p_fail", C.c_double), ("p_info", C.c_double),
                ("n_bad_reads", C.c_int64), ("seed", C.c_uint64)]


class _SetParams(C.Structure):
    _fields_ = [("n_adds", C.c_int64), ("n_procs", C.c_int32), ("pad", C.c_int32),
                ("p_fail", C.c_double), ("p_info", C.c_double),
                ("n_lost", C.c_int64), ("n_unexpected", C.c_int64), ("seed", C.c_uint64)]


_p64 = C.POINTER(C.c_int64)


class _Hist(C.Structure):
    _fields_ = [("n", C.c_int64), ("n_aux", C.c_int64), ("n_keys", C.c_int64),
                ("process", _p64), ("type", _p64), ("f", _p64), ("key", _p64),
                ("value", _p64), ("value2", _p64), ("aux", _p64), ("truth", _p64),
                ("impl", C.c_void_p)]


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libjhgen.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        _lib = C.CDLL(path)
        _lib.jhg_cas.argtypes = [C.POINTER(_CasParams), C.POINTER(_Hist)]
        _lib.jhg_cas_par.argtypes = [C.POINTER(_CasParams), C.c_int32, C.POINTER(_Hist)]
        _lib.jhg_counter.argtypes = [C.POINTER(_CounterParams), C.POINTER(_Hist)]
        _lib.jhg_set.argtypes = [C.POINTER(_SetParams), C.POINTER(_Hist)]
        _lib.jhg_free.argtypes = [C.POINTER(_Hist)]
    return _lib


def _take(h, n_truth):
    def arr(p, n):
        if n == 0:
            return np.zeros(0, np.int64)
        return np.ctypeslib.as_array(p, shape=(n,)).copy()
    n = h.n
    cols = Columns(n=n, process=arr(h.process, n), type=arr(h.type, n), f=arr(h.f, n),
                   key=arr(h.key, n), value=arr(h.value, n), value2=arr(h.value2, n),
                   n_keys=h.n_keys,
                   aux=arr(h.aux, h.n_aux) if h.n_aux else np.zeros(1, np.int64))
    cols.keys = list(range(h.n_keys))
    cols.f_names = ["start", "stop"]
    truth = arr(h.truth, n_truth) if n_truth else np.zeros(0, np.int64)
    return cols, truth


def cas_register(n_keys=10000, ops_per_key=500, threads_per_key=10, readers=5,
                 n_values=5, process_limit=20, groups=10, init_nil=True,
                 p_info=0.02, p_invalid=0.01, nemesis_every=10000, seed=3, keyed=True, parts=1):
    """Independent cas-register history (C3 defaults: 10k keys x ~1k entries).

    parts > 1 generates the keys as that many sub-histories on parallel host
    threads and concatenates them (gen.cpp jhg_cas_par; the C4 1M-key history).
    Returns (Columns, injected) where injected[k] = 1 for keys with a
    stale read injected (all other keys are linearizable by construction)."""
    lib = _load()
    p = _CasParams(n_keys, ops_per_key, threads_per_key, readers, n_values, process_limit,
                   groups, 1 if init_nil else 0, p_info, p_invalid, nemesis_every, seed,
                   1 if keyed else 0, 0)
    h = _Hist()
    if parts > 1:
        lib.jhg_cas_par(C.byref(p), parts, C.byref(h))
    else:
        lib.jhg_cas(C.byref(p), C.byref(h))
    try:
        return _take(h, n_keys)
    finally:
        lib.jhg_free(C.byref(h))


def counter(n_ops=1000, n_procs=10, read_every=101, p_fail=0.05, p_info=0.01,
            n_bad_reads=0, seed=2):
    lib = _load()
    p = _CounterParams(n_ops, n_procs, read_every, p_fail, p_info, n_bad_reads, seed)
    h = _Hist()
    lib.jhg_counter(C.byref(p), C.byref(h))
    try:
        return _take(h, 0)[0]
    finally:
        lib.jhg_free(C.byref(h))


def set_history(n_adds=1000, n_procs=10, p_fail=0.05, p_info=0.02, n_lost=0,
                n_unexpected=0, seed=2):
    lib = _load()
    p = _SetParams(n_adds, n_procs, 0, p_fail, p_info, n_lost, n_unexpected, seed)
    h = _Hist()
    lib.jhg_set(C.byref(p), C.byref(h))
    try:
        return _take(h, 0)[0]
    finally:
        lib.jhg_free(C.byref(h))


def set_full_history(n_adds=2000, n_procs=10, n_readers=2, read_every=10, p_fail=0.05,
                     p_info=0.02, n_lost=0, n_stale=0, row_ns=100_000, seed=6):
    """A (checker/set-full) workload (checker.clj:236-534; the shape of
    yugabyte/src/yugabyte/set.clj:92 and tidb/src/tidb/sets.clj:53): adds of
    distinct integers 0..n_adds-1 by `n_procs` processes, `n_readers`
    processes reading the WHOLE set every `read_every` rounds of adds.

    A round invokes one add per process and completes them in random order;
    a read invoked before a round completes after it. :ok adds are visible
    from their completion on, adds concurrent with a read are seen with
    probability 1/2, :info adds apply with probability 1/2 (and rename the
    process, core.clj:349), :fail adds never apply. Faults: `n_lost`
    acknowledged elements vanish from every read after the middle of the
    history (lost), `n_stale` elements are missed by the first read invoked
    after their :ok (stale, stable latency > 0). :time = row * row_ns.

    Returns (Columns, time) with the set reads' elements in `aux` (CSR)."""
    rng = np.random.default_rng(seed)
    P, RD = n_procs, n_readers
    rows_p, rows_t, rows_f, rows_v, rows_v2 = [], [], [], [], []
    aux_parts, aux_len = [], 0
    applied = np.zeros(n_adds, bool)          # visible from completion on
    acked_row = np.full(n_adds, -1, np.int64)
    proc_id = list(range(P))
    next_proc = P + RD
    n_rounds = (n_adds + P - 1) // P
    lost = rng.choice(n_adds, size=n_lost, replace=False) if n_lost else np.zeros(0, np.int64)
    stale = set(rng.choice(n_adds, size=n_stale, replace=False).tolist()) if n_stale else set()
    stale_pending = []
    reader = 0
    mid_round = n_rounds // 2

    def emit(p, t, f, v=JH_NIL, v2=JH_NIL):
        rows_p.append(p); rows_t.append(t); rows_f.append(f); rows_v.append(v); rows_v2.append(v2)

    for k in range(n_rounds):
        els = list(range(k * P, min(n_adds, (k + 1) * P)))
        rd = (k % read_every) == read_every - 1
        if rd:
            rp = P + (reader % RD)
            reader += 1
            emit(rp, 0, 0)                     # :invoke :read
            hide, stale_pending = stale_pending, []   # acked before this read's invocation
        for j, e in enumerate(els):
            emit(proc_id[j], 0, 3, e)          # :invoke :add e
        outcome = rng.random(len(els))
        seen_conc = rng.random(len(els)) < 0.5
        for j in rng.permutation(len(els)):
            e = els[j]
            if outcome[j] < p_fail:
                emit(proc_id[j], 2, 3, e)
            elif outcome[j] < p_fail + p_info:
                emit(proc_id[j], 3, 3, e)
                applied[e] = rng.random() < 0.5
                proc_id[j] = next_proc
                next_proc += 1
            else:
                applied[e] = True
                acked_row[e] = len(rows_p)
                emit(proc_id[j], 1, 3, e)
                if e in stale:
                    stale_pending.append(e)
        if rd:
            vis = applied.copy()
            conc = np.asarray(els, np.int64)
            vis[conc] = applied[conc] & seen_conc
            if k >= mid_round and n_lost:
                vis[lost] = False
            for e in hide:
                vis[e] = False
            elems = np.flatnonzero(vis).astype(np.int64)
            emit(rp, 1, 0, aux_len, len(elems))
            aux_parts.append(elems)
            aux_len += len(elems)
    n = len(rows_p)
    cols = Columns(n=n, process=np.asarray(rows_p, np.int64), type=np.asarray(rows_t, np.int64),
                   f=np.asarray(rows_f, np.int64), key=np.full(n, -1, np.int64),
                   value=np.asarray(rows_v, np.int64), value2=np.asarray(rows_v2, np.int64),
                   n_keys=0, aux=np.concatenate(aux_parts) if aux_parts else np.zeros(1, np.int64))
    time = np.arange(n, dtype=np.int64) * row_ns
    return cols, time


def columns_to_ops(cols, time):
    """Op maps (jepsen_amd.history form) of a set-full Columns history, for the
    pure-Python oracle and the checker mirror."""
    names = {0: "invoke", 1: "ok", 2: "fail", 3: "info"}
    fnames = {0: "read", 3: "add"}
    ops = []
    for i in range(cols.n):
        t, f = int(cols.type[i]), int(cols.f[i])
        if f == 0 and t == 1:
            o, c = int(cols.value[i]), int(cols.value2[i])
            v = cols.aux[o:o + c].tolist()
        elif f == 0:
            v = None
        else:
            v = int(cols.value[i])
        ops.append({"process": int(cols.process[i]), "type": names[t], "f": fnames[f],
                    "value": v, "index": i, "time": int(time[i])})
    return ops


def queue_history(n_enqueues=2000, n_procs=5, p_fail=0.05, p_info=0.05, n_lost=0, n_unexpected=0,
                  n_duplicated=0, n_repeat=0, drain_parts=2, seed=7):
    """A queue workload for (checker/total-queue) and (checker/queue
    (model/unordered-queue)) (checker.clj:160-180, 536-628; the shape of
    disque.clj:305-309 and rabbitmq_test.clj:56-59): `n_procs` enqueuers, one
    dequeuer taking a random pending element after every round, and a final
    drain in `drain_parts` :drain ops. Values are consecutive integers (as
    gen/queue, generator.clj:405-416) except `n_repeat` values enqueued twice. :fail enqueues never apply, :info ones
    apply with probability 1/2. Faults: `n_lost` acknowledged elements are
    never dequeued, `n_unexpected` never-enqueued values are dequeued,
    `n_duplicated` elements are dequeued twice. Returns Columns (drain
    elements in aux)."""
    rng = np.random.default_rng(seed)
    P = n_procs
    DQ = P                                  # dequeuer process
    # consecutive integers, as gen/queue enqueues them (generator.clj:405-416)
    vals = np.arange(n_enqueues, dtype=np.int64)
    if n_repeat:
        vals[-n_repeat:] = vals[:n_repeat]
    rows = []
    aux = []
    pending = []                            # applied, not yet dequeued
    lost_left = n_lost
    proc_id = list(range(P))
    next_proc = P + 1
    dup_left = n_duplicated
    dequeued = []
    for k in range(0, n_enqueues, P):
        els = vals[k:k + P]
        for j, v in enumerate(els):
            rows.append((proc_id[j], 0, 4, int(v), JH_NIL))
        for j in rng.permutation(len(els)):
            v = int(els[j])
            u = rng.random()
            if u < p_fail:
                rows.append((proc_id[j], 2, 4, v, JH_NIL))
            elif u < p_fail + p_info:
                rows.append((proc_id[j], 3, 4, v, JH_NIL))
                proc_id[j] = next_proc
                next_proc += 1
                if rng.random() < 0.5:
                    pending.append(v)
            else:
                rows.append((proc_id[j], 1, 4, v, JH_NIL))
                if lost_left and rng.random() < 0.3:
                    lost_left -= 1          # acknowledged, then lost
                else:
                    pending.append(v)
        if pending:
            i = int(rng.integers(len(pending)))
            v = pending.pop(i)
            rows.append((DQ, 0, 5, JH_NIL, JH_NIL))
            rows.append((DQ, 1, 5, v, JH_NIL))
            dequeued.append(v)
            if dup_left and rng.random() < 0.2:
                dup_left -= 1
                rows.append((DQ, 0, 5, JH_NIL, JH_NIL))
                rows.append((DQ, 1, 5, v, JH_NIL))
    rest = pending + [int(x) for x in dequeued[:dup_left]]
    rest += [int(n_enqueues + 100 + i) for i in range(n_unexpected)]
    rng.shuffle(rest)
    parts = np.array_split(np.asarray(rest, np.int64), max(drain_parts, 1))
    for part in parts:
        rows.append((DQ, 0, 6, JH_NIL, JH_NIL))
        rows.append((DQ, 1, 6, len(aux), len(part)))
        aux.extend(part.tolist())
    a = np.asarray(rows, np.int64).reshape(-1, 5)
    n = len(a)
    return Columns(n=n, process=a[:, 0].copy(), type=a[:, 1].copy(), f=a[:, 2].copy(),
                   key=np.full(n, -1, np.int64), value=a[:, 3].copy(), value2=a[:, 4].copy(),
                   n_keys=0, aux=np.asarray(aux, np.int64) if aux else np.zeros(1, np.int64))


def queue_columns_to_ops(cols):
    """Op maps of a queue_history (for the oracles and the checker mirror)."""
    names = {0: "invoke", 1: "ok", 2: "fail", 3: "info"}
    fnames = {4: "enqueue", 5: "dequeue", 6: "drain"}
    ops = []
    for i in range(cols.n):
        t, f = int(cols.type[i]), int(cols.f[i])
        v = int(cols.value[i])
        if f == 6 and t == 1:
            val = cols.aux[v:v + int(cols.value2[i])].tolist()
        else:
            val = None if v == JH_NIL else v
        ops.append({"process": int(cols.process[i]), "type": names[t], "f": fnames[f], "value": val})
    return ops
