"""Seeded synthetic histories from libjhgen.so.

Workload generator for bench.py and the tests: the histories are shaped like
the reference workloads (see csrc/gen.cpp header) and are returned as
`history.Columns` (host numpy int64 columns in the include/jh.h layout).
"""
import ctypes as C
import os

import numpy as np

from .history import Columns

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
                 p_info=0.02, p_invalid=0.01, nemesis_every=10000, seed=3, keyed=True):
    """Independent cas-register history (C3 defaults: 10k keys x ~1k entries).

    Returns (Columns, injected) where injected[k] = 1 for keys with a
    stale read injected (all other keys are linearizable by construction)."""
    lib = _load()
    p = _CasParams(n_keys, ops_per_key, threads_per_key, readers, n_values, process_limit,
                   groups, 1 if init_nil else 0, p_info, p_invalid, nemesis_every, seed,
                   1 if keyed else 0, 0)
    h = _Hist()
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
