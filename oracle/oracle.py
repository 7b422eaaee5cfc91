"""TEST INFRASTRUCTURE ONLY: ctypes wrapper around oracle/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline. The product
path (jepsen_amd + libjh.so) never imports it.

See jh_oracle.h for what the oracle restates and how it is pinned.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from jepsen_amd import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def build(quiet=True):
    subprocess.run(["make", "-C", _HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        H = C.POINTER(A.JhHistory)
        V = C.POINTER(A.JhKeyVerdict)
        p64 = C.POINTER(C.c_int64)
        L.orc_check_cas.argtypes = [H, C.c_int64, C.c_int64, V]
        L.orc_check_cas_independent.argtypes = [H, C.c_int64, C.c_int64, C.c_int, C.c_int, V,
                                                C.POINTER(A.JhSummary)]
        L.orc_check_cas_independent_range.argtypes = [H, C.c_int64, C.c_int64, C.c_int, C.c_int,
                                                      C.c_int64, C.c_int64, V]
        L.orc_check_counter.argtypes = [H, p64, C.c_int64, p64, p64, p64,
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.orc_check_set.argtypes = [H, C.POINTER(A.JhSetResult), p64, p64, p64, p64, C.c_int64]
        L.orc_interval_str.argtypes = [p64, C.c_int64, C.c_char_p, C.c_int64]
        L.orc_interval_str.restype = C.c_int64
        L.orc_lin_selftest_key.argtypes = [H, C.c_int64, C.c_int64, p64]
        L.orc_lin_configs.argtypes = [H, C.c_int64, C.c_int64, p64, C.c_int64, C.c_int32, C.c_int32,
                                      C.POINTER(A.JhLinConfig), C.POINTER(C.c_int32), p64]
        _lib = L
    return _lib


def check_cas(cols, init=A.NIL, budget=A.DEFAULT_BUDGET):
    h = cols.as_jh()
    v = A.JhKeyVerdict()
    lib().orc_check_cas(C.byref(h), init, budget, C.byref(v))
    return v.valid, v.cause, v.fail_entry, v.explored


def check_cas_full(cols, init=A.NIL, budget=A.DEFAULT_BUDGET):
    h = cols.as_jh()
    v = A.JhKeyVerdict()
    lib().orc_check_cas(C.byref(h), init, budget, C.byref(v))
    return {f: getattr(v, f) for f, _ in A.JhKeyVerdict._fields_}


def linear_states_ok(cols, init=A.NIL):
    """The device's history-wide condition for the reachable-set engine (every
    interned state id < 4096): the value range of client read / write / cas
    ops (and the initial value) when it is interned as one range, else the
    largest number of distinct values of one key (per-key interning)."""
    cl = (cols.process >= 0) & (cols.f <= A.F_CAS)
    v = cols.value[cl]
    v2 = cols.value2[cl & (cols.f == A.F_CAS)] if cols.n else cols.value2[:0]
    vals = np.concatenate([v[v != A.NIL], v2[v2 != A.NIL]] + ([np.array([init])] if init != A.NIL else []))
    if len(vals) == 0:
        return True
    if int(vals.max()) - int(vals.min()) < 0xFFFE - 3:
        return int(vals.max()) - int(vals.min()) + 2 < 4096
    keys = cols.key[cl] if cols.key is not None else np.zeros(int(cl.sum()), np.int64)
    worst = 0
    for k in np.unique(keys):
        sel = cl.copy()
        sel[cl] = keys == k
        a = cols.value[sel]
        b = cols.value2[sel & (cols.f == A.F_CAS)]
        d = len(np.unique(np.concatenate([a[a != A.NIL], b[b != A.NIL]] + ([np.array([init])] if init != A.NIL else []))))
        worst = max(worst, d)
    return worst + 1 < 4096


def check_cas_independent(cols, init=A.NIL, budget=A.DEFAULT_BUDGET, mode=0, threads=1, algorithm=None):
    """Returns (verdicts structured array [n_keys], summary). algorithm
    "linear": JIT linearization where the device's reachable-set engine
    applies (mode bit 2), WGL elsewhere, with each key's :analyzer."""
    if algorithm == "linear":
        mode |= 4
        C.c_int.in_dll(lib(), "orc_linear_states_ok").value = 1 if linear_states_ok(cols, init) else 0
    h = cols.as_jh()
    out = np.zeros(max(cols.n_keys, 1), dtype=A.VERDICT_DTYPE)
    s = A.JhSummary()
    lib().orc_check_cas_independent(C.byref(h), init, budget, mode, threads,
                                    out.ctypes.data_as(C.POINTER(A.JhKeyVerdict)), C.byref(s))
    return out[:cols.n_keys], s


def per_key_values(cols, init=A.NIL):
    """Whether the device numbers register values per key (their range spans
    more than one 16-bit state range)."""
    cl = (cols.process >= 0) & (cols.f <= A.F_CAS)
    v = cols.value[cl]
    v2 = cols.value2[cl & (cols.f == A.F_CAS)]
    vals = np.concatenate([v[v != A.NIL], v2[v2 != A.NIL]] + ([np.array([init])] if init != A.NIL else []))
    return len(vals) > 0 and int(vals.max()) - int(vals.min()) >= 0xFFFE - 3


def lin_configs(cols, keys, per_key=A.CONFIGS_PER_KEY, init=A.NIL, budget=A.DEFAULT_BUDGET):
    """orc_lin_configs, the restatement of jh_lin_configs (same return shape
    as _native.Context.lin_configs)."""
    C.c_int.in_dll(lib(), "orc_linear_states_ok").value = 1 if linear_states_ok(cols, init) else 0
    h = cols.as_jh()
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
    nq = len(keys)
    out = (A.JhLinConfig * max(nq * per_key, 1))()
    n_out = np.zeros(max(nq, 1), np.int32)
    rows = np.zeros(max(nq * per_key * A.MAX_WINDOW, 1), np.int64)
    lib().orc_lin_configs(C.byref(h), init, budget, A.ptr64(keys), nq, per_key,
                          1 if per_key_values(cols, init) else 0, out,
                          n_out.ctypes.data_as(C.POINTER(C.c_int32)), A.ptr64(rows))
    res = {}
    for i, k in enumerate(keys.tolist()):
        if n_out[i] < 0:
            res[k] = None
            continue
        cs = []
        for j in range(n_out[i]):
            c = out[i * per_key + j]
            r = rows[c.rows_off:c.rows_off + c.n_linearized + c.n_pending]
            cs.append((int(c.model_value), r[:c.n_linearized].tolist(), r[c.n_linearized:].tolist(),
                       int(c.last_row)))
        res[k] = cs
    return res


def check_cas_independent_range(cols, k0, k1, init=A.NIL, budget=A.DEFAULT_BUDGET, mode=0,
                                threads=1):
    h = cols.as_jh()
    out = np.zeros(max(k1 - k0, 1), dtype=A.VERDICT_DTYPE)
    lib().orc_check_cas_independent_range(C.byref(h), init, budget, mode, threads, k0, k1,
                                          out.ctypes.data_as(C.POINTER(A.JhKeyVerdict)))
    return out[:k1 - k0]


def key_selftest(cols, init=A.NIL, budget=A.DEFAULT_BUDGET):
    """Runs the three CPU formulations on a whole (single-key) history.

    Returns dict with canonical/list/bruteforce verdicts and explored counts."""
    h = cols.as_jh()
    res = np.zeros(8, np.int64)
    lib().orc_lin_selftest_key(C.byref(h), init, budget, A.ptr64(res))
    return {"status": int(res[0]), "canonical": int(res[1]), "canonical_explored": int(res[2]),
            "list": int(res[3]), "list_explored": int(res[4]), "bruteforce": int(res[5]),
            "n_ops": int(res[6]), "max_window": int(res[7])}


def check_counter(cols, reads_cap=None):
    h = cols.as_jh()
    cap = cols.n if reads_cap is None else reads_cap
    reads = np.zeros(3 * max(cap, 1), np.int64)
    nr, ne, fe = C.c_int64(), C.c_int64(), C.c_int64()
    valid, cause = C.c_int32(), C.c_int32()
    lib().orc_check_counter(C.byref(h), A.ptr64(reads), cap, C.byref(nr), C.byref(ne),
                            C.byref(fe), C.byref(valid), C.byref(cause))
    k = min(nr.value, cap)
    return {"valid": valid.value, "cause": cause.value, "reads": reads[:3 * k].reshape(-1, 3),
            "n_reads": nr.value, "n_errors": ne.value, "first_err_entry": fe.value}


def check_set(cols, runs_cap=None):
    h = cols.as_jh()
    cap = (cols.n + len(cols.aux) + 2) if runs_cap is None else runs_cap
    runs = [np.zeros(2 * max(cap, 1), np.int64) for _ in range(4)]
    r = A.JhSetResult()
    lib().orc_check_set(C.byref(h), C.byref(r), *[A.ptr64(x) for x in runs], cap)
    out = {name: getattr(r, name) for name, _ in A.JhSetResult._fields_ if name != "n_runs"}
    out["runs"] = [runs[i][:2 * min(r.n_runs[i], cap)].reshape(-1, 2) for i in range(4)]
    out["n_runs"] = list(r.n_runs)
    return out


def interval_str(values):
    a = np.asarray(sorted(set(int(x) for x in values)), np.int64)
    buf = C.create_string_buffer(64 + 24 * max(len(a), 1))
    lib().orc_interval_str(A.ptr64(a) if len(a) else None, len(a), buf, len(buf))
    return buf.value.decode()
