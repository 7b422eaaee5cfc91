"""ctypes binding of libjh.so (include/jh.h). The product path: there is no
CPU fallback. If the library or a GPU is missing, every call raises.
"""
import ctypes as C
import os
import threading

import numpy as np

from . import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JH_LIB") or os.path.join(_HERE, "libjh.so")   # JH_LIB: A/B builds (tools/)
_lib = None
_lock = threading.Lock()


class JhError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libjh error {code}: {msg}")
        self.code = code
        self.msg = msg


def lib():
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"{LIB_PATH} is missing: run `python -m jepsen_amd.build` "
                                   "(the HIP extension is required; there is no CPU fallback)")
            L = C.CDLL(LIB_PATH)
            H = C.POINTER(A.JhHistory)
            L.jh_version.restype = C.c_int
            L.jh_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
            L.jh_open_multi.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
            L.jh_open_devices.argtypes = [C.POINTER(C.c_int32), C.c_int, C.POINTER(C.c_void_p)]
            L.jh_n_devices.argtypes = [C.c_void_p]
            L.jh_key_index.argtypes = [C.c_void_p, H, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                       C.c_char_p, C.c_size_t]
            L.jh_key_costs.argtypes = [C.POINTER(A.JhHistory), C.POINTER(C.c_int64), C.c_char_p, C.c_size_t]
            L.jh_stage_history.argtypes = [C.c_void_p, H, C.POINTER(C.c_int64), C.c_char_p, C.c_size_t]
            L.jh_close.argtypes = [C.c_void_p]
            L.jh_close.restype = None
            L.jh_check_cas_independent.argtypes = [C.c_void_p, H, C.POINTER(A.JhLinOpts),
                                                   C.POINTER(A.JhKeyVerdict), C.POINTER(A.JhSummary),
                                                   C.c_char_p, C.c_size_t]
            L.jh_check_cas_independent_device.argtypes = L.jh_check_cas_independent.argtypes
            L.jh_lin_configs.argtypes = [C.c_void_p, H, C.POINTER(A.JhLinOpts), C.POINTER(C.c_int64), C.c_int64,
                                         C.c_int32, C.POINTER(A.JhLinConfig), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int64), C.c_int64, C.c_char_p, C.c_size_t]
            L.jh_check_cas.argtypes = [C.c_void_p, H, C.POINTER(A.JhLinOpts),
                                       C.POINTER(A.JhKeyVerdict), C.c_char_p, C.c_size_t]
            p64 = C.POINTER(C.c_int64)
            L.jh_check_counter.argtypes = [C.c_void_p, H, p64, C.c_int64, p64, p64, p64,
                                           C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                           C.c_char_p, C.c_size_t]
            L.jh_check_set.argtypes = [C.c_void_p, H, C.POINTER(A.JhSetResult), p64, p64, p64, p64,
                                       C.c_int64, C.c_char_p, C.c_size_t]
            p32 = C.POINTER(C.c_uint32)
            L.jh_check_set_bitmaps.argtypes = [C.c_void_p, H, C.POINTER(A.JhSetResult), p32, p32, p32, p32,
                                               C.c_int64, p64, p64, C.c_char_p, C.c_size_t]
            L.jh_check_set_full.argtypes = [C.c_void_p, H, p64, C.c_int32, C.POINTER(A.JhSetFullResult),
                                            p64, p64, p64, C.c_int64, C.c_char_p, C.c_size_t]
            L.jh_check_set_full_opts.argtypes = [C.c_void_p, H, p64, C.POINTER(A.JhSetFullOpts),
                                                 C.POINTER(A.JhSetFullResult), p64, p64, p64, C.c_int64,
                                                 C.c_char_p, C.c_size_t]
            L.jh_check_total_queue.argtypes = [C.c_void_p, H, C.POINTER(A.JhQueueResult), p64, p64, p64, p64,
                                               C.c_int64, C.c_char_p, C.c_size_t]
            L.jh_check_queue.argtypes = [C.c_void_p, H, C.POINTER(A.JhQueueResult), p64, C.c_int64,
                                         C.c_char_p, C.c_size_t]
            L.jh_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p), C.c_char_p, C.c_size_t]
            L.jh_host_free.argtypes = [C.c_void_p]
            # history ingest (include/jh_io.h), host code in the same library
            pp = C.POINTER(C.c_void_p)
            L.jh_ingest_file.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, pp, C.c_char_p, C.c_size_t]
            L.jh_ingest_buffer.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.c_int, pp,
                                           C.c_char_p, C.c_size_t]
            io = C.POINTER(A.JhIngestOpts)
            L.jh_ingest_file_opts.argtypes = [C.c_char_p, C.c_int, C.c_int, io, pp, C.c_char_p, C.c_size_t]
            L.jh_ingest_buffer_opts.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, io, pp,
                                                C.c_char_p, C.c_size_t]
            L.jh_ingest_history.argtypes = [C.c_void_p, H]
            L.jh_ingest_history.restype = None
            L.jh_ingest_time.argtypes = [C.c_void_p]
            L.jh_ingest_time.restype = p64
            L.jh_ingest_values_interned.argtypes = [C.c_void_p]
            L.jh_ingest_table_size.argtypes = [C.c_void_p, C.c_int]
            L.jh_ingest_table_size.restype = C.c_int64
            L.jh_ingest_table_entry.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_char_p, C.c_size_t]
            L.jh_ingest_table_entry.restype = C.c_int64
            L.jh_ingest_free.argtypes = [C.c_void_p]
            L.jh_ingest_free.restype = None
            if L.jh_version() != A.JH_ABI_VERSION:
                raise RuntimeError("libjh.so ABI version mismatch")
            _lib = L
    return _lib


EXPORTED_SYMBOLS = ["jh_version", "jh_open", "jh_open_multi", "jh_open_devices", "jh_n_devices", "jh_key_costs", "jh_key_index",
                    "jh_stage_history",
                    "jh_close", "jh_check_cas_independent",
                    "jh_check_cas", "jh_check_cas_independent_device", "jh_lin_configs", "jh_check_counter",
                    "jh_check_set", "jh_check_set_bitmaps", "jh_check_set_full", "jh_check_set_full_opts", "jh_check_total_queue", "jh_check_queue",
                    "jh_host_alloc", "jh_host_free",
                    # include/jh_io.h
                    "jh_ingest_file", "jh_ingest_buffer", "jh_ingest_file_opts", "jh_ingest_buffer_opts", "jh_ingest_history", "jh_ingest_time",
                    "jh_ingest_values_interned", "jh_ingest_table_size", "jh_ingest_table_entry", "jh_ingest_free"]


def _raise(rc, err):
    if rc != A.JH_OK:
        raise JhError(rc, err.value.decode(errors="replace"))


def _opts(init, budget, stream=0, algorithm=None, exact_count=True, **tune):
    """jh_lin_opts. tune: flags, quick_budget, phase2_budget, helpers,
    helper_late_us, xw_waves, p2_waves_per_cu (jh.h; all decide the same
    verdicts, the tests use them to reach the less common search paths).
    exact_count: JH_LIN_EXACT_COUNT, WGL's cache size for every key (what the
    parity tests compare with the oracle); the checkers pass False -- their
    result maps carry no :explored, and the count pass then leaves the
    critical path."""
    o = A.JhLinOpts()
    o.init_value = A.NIL if init is None else int(init)
    o.budget = int(budget or 0)
    o.stream = int(stream)
    if isinstance(algorithm, str):
        algorithm = A.ALGORITHMS[algorithm]
    o.algorithm = int(algorithm or 0)
    for k, v in tune.items():
        if k not in dict(A.JhLinOpts._fields_) or k in ("init_value", "budget", "stream", "algorithm", "reserved", "reserved2"):
            raise TypeError(f"unknown jh_lin_opts field {k}")
        setattr(o, k, int(v))
    if exact_count:
        o.flags |= A.LIN_EXACT_COUNT
    return o


def key_costs(cols):
    """jh_key_costs: per-key search-cost estimate (entries + window sum), the
    weight that splits keys between devices. Host-only: needs no GPU."""
    h = A.make_history(cols)
    out = np.zeros(max(cols.n_keys, 1), dtype=np.int64)
    err = C.create_string_buffer(256)
    rc = lib().jh_key_costs(C.byref(h), out.ctypes.data_as(C.POINTER(C.c_int64)), err, len(err))
    _raise(rc, err)
    return out[:cols.n_keys]


class HostBuffer:
    """Page-locked host memory from jh_host_alloc, viewed as a numpy array:
    result buffers reused across calls (check_counter's reads, the set
    bitmaps), so their D2H runs at PCIe speed. Freed with the object."""

    def __init__(self, count, dtype):
        dt = np.dtype(dtype)
        p = C.c_void_p()
        err = C.create_string_buffer(256)
        _raise(lib().jh_host_alloc(max(int(count), 1) * dt.itemsize, C.byref(p), err, len(err)), err)
        self._p = p
        buf = (C.c_char * (max(int(count), 1) * dt.itemsize)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dt, count=max(int(count), 1))

    def __del__(self):
        p = getattr(self, "_p", None)
        if p is not None and p.value:
            self.array = None
            lib().jh_host_free(p)
            self._p = None


class Context:
    """One jh_ctx on one HIP device (jh_open / jh_close), or, with n_gpus, one
    context over devices 0..n_gpus-1 (jh_open_multi: the independent check is
    split by key over them inside libjh)."""

    def __init__(self, device=0, n_gpus=None, devices=None):
        L = lib()
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int32 * len(devices))(*devices)
            rc = L.jh_open_devices(arr, len(devices), C.byref(h))
        elif n_gpus is None:
            rc = L.jh_open(int(device), C.byref(h))
        else:
            rc = L.jh_open_multi(int(n_gpus), C.byref(h))
        if rc != A.JH_OK:
            raise JhError(rc, f"jh_open({device}, n_gpus={n_gpus}) failed (no usable HIP device?)")
        self._h = h
        self.device = device
        self.n_devices = L.jh_n_devices(h)

    def close(self):
        if getattr(self, "_h", None):
            lib().jh_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def key_index(self, cols):
        """jh_key_index: (key_off [n_keys+1], rows [n]) -- key k's rows are
        rows[key_off[k]:key_off[k+1]] in history order, the un-keyed rows
        rows[key_off[n_keys]:]."""
        h = A.make_history(cols)
        off = np.zeros(cols.n_keys + 1, np.int64)
        rows = np.zeros(max(cols.n, 1), np.int64)
        err = C.create_string_buffer(512)
        p64 = C.POINTER(C.c_int64)
        rc = lib().jh_key_index(self._h, C.byref(h), off.ctypes.data_as(p64), rows.ctypes.data_as(p64),
                                err, len(err))
        _raise(rc, err)
        return off, rows[:cols.n]

    def stage_history(self, cols):
        """jh_stage_history: the six int64 columns (process, type, f, key,
        value, value2) as the device holds them after staging the host
        history -- the packed path for >= 2 M rows (jh_ingest.hip)."""
        h = A.make_history(cols)
        out = np.zeros(6 * max(cols.n, 1), np.int64)
        err = C.create_string_buffer(512)
        _raise(lib().jh_stage_history(self._h, C.byref(h), A.ptr64(out), err, len(err)), err)
        return out[:6 * cols.n].reshape(6, cols.n)

    # -- linearizability ---------------------------------------------------
    def check_cas_independent(self, cols, init=None, budget=None, **tune):
        """Returns (verdicts: structured array [n_keys] of VERDICT_DTYPE, JhSummary)."""
        h = A.make_history(cols)
        out = np.zeros(max(cols.n_keys, 1), dtype=A.VERDICT_DTYPE)
        s = A.JhSummary()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_cas_independent(self._h, C.byref(h), C.byref(_opts(init, budget, **tune)),
                                            out.ctypes.data_as(C.POINTER(A.JhKeyVerdict)),
                                            C.byref(s), err, len(err))
        _raise(rc, err)
        return out[:cols.n_keys], s

    def check_cas_independent_device(self, dcols, verdicts_dev_ptr, init=None, budget=None,
                                     stream=0, **tune):
        """dcols: object whose column attributes are device pointers (ints)."""
        h = A.make_history(dcols, on_device=True)
        s = A.JhSummary()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_cas_independent_device(
            self._h, C.byref(h), C.byref(_opts(init, budget, stream, **tune)),
            C.cast(C.c_void_p(int(verdicts_dev_ptr)), C.POINTER(A.JhKeyVerdict)),
            C.byref(s), err, len(err))
        _raise(rc, err)
        return s

    def check_cas(self, cols, init=None, budget=None, **tune):
        h = A.make_history(cols)
        v = A.JhKeyVerdict()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_cas(self._h, C.byref(h), C.byref(_opts(init, budget, **tune)), C.byref(v),
                                err, len(err))
        _raise(rc, err)
        return v.valid, v.cause, v.fail_entry, v.explored

    def check_cas_full(self, cols, init=None, budget=None, **tune):
        """jh_check_cas -> {valid, cause, fail_entry, explored, previous_ok, last_op}."""
        h = A.make_history(cols)
        v = A.JhKeyVerdict()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_cas(self._h, C.byref(h), C.byref(_opts(init, budget, **tune)), C.byref(v),
                                err, len(err))
        _raise(rc, err)
        return {f: getattr(v, f) for f, _ in A.JhKeyVerdict._fields_}

    def lin_configs(self, cols, keys, per_key=A.CONFIGS_PER_KEY, init=None, budget=None, **tune):
        """jh_lin_configs: {key: None | [(model_value, linearized rows, pending rows, last_row)]}
        -- each invalid key's frontier, each valid :linear key's final
        configurations (include/jh.h)."""
        h = A.make_history(cols)
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
        nq = len(keys)
        out = (A.JhLinConfig * max(nq * per_key, 1))()
        n_out = np.zeros(max(nq, 1), np.int32)
        rows = np.zeros(max(nq * per_key * A.MAX_WINDOW, 1), np.int64)
        err = C.create_string_buffer(1024)
        rc = lib().jh_lin_configs(self._h, C.byref(h), C.byref(_opts(init, budget, **tune)),
                                  keys.ctypes.data_as(C.POINTER(C.c_int64)), nq, per_key, out,
                                  n_out.ctypes.data_as(C.POINTER(C.c_int32)), A.ptr64(rows), len(rows),
                                  err, len(err))
        _raise(rc, err)
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

    # -- counter / set -----------------------------------------------------
    def check_counter(self, cols, reads_cap=None, on_device=False, out=None):
        """on_device: cols' columns are device pointers (the history already in HBM).
        out: an int64 array of >= 3 * reads_cap to receive the triples (e.g. a
        HostBuffer's, reused across calls); the returned reads view it."""
        h = A.make_history(cols, on_device=on_device)
        cap = cols.n if reads_cap is None else reads_cap
        if out is not None:
            if out.dtype != np.int64 or len(out) < 3 * max(cap, 1) or not out.flags.c_contiguous:
                raise ValueError("out: contiguous int64 array of at least 3 * reads_cap")
            reads = out
        else:
            reads = np.zeros(3 * max(cap, 1), np.int64)
        nr, ne, fe = C.c_int64(), C.c_int64(), C.c_int64()
        valid, cause = C.c_int32(), C.c_int32()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_counter(self._h, C.byref(h), A.ptr64(reads), cap, C.byref(nr),
                                    C.byref(ne), C.byref(fe), C.byref(valid), C.byref(cause),
                                    err, len(err))
        _raise(rc, err)
        k = min(nr.value, cap)
        return {"valid": valid.value, "cause": cause.value, "reads": reads[:3 * k].reshape(-1, 3),
                "n_reads": nr.value, "n_errors": ne.value, "first_err_entry": fe.value}

    def check_set(self, cols, runs_cap=None, on_device=False):
        h = A.make_history(cols, on_device=on_device)
        n_aux = int(cols.n_aux) if on_device else len(cols.aux)
        cap = (cols.n + n_aux + 2) if runs_cap is None else runs_cap
        runs = [np.zeros(2 * max(cap, 1), np.int64) for _ in range(4)]
        r = A.JhSetResult()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_set(self._h, C.byref(h), C.byref(r), *[A.ptr64(x) for x in runs], cap,
                                err, len(err))
        _raise(rc, err)
        out = {name: getattr(r, name) for name, _ in A.JhSetResult._fields_ if name != "n_runs"}
        out["runs"] = [runs[i][:2 * min(r.n_runs[i], cap)].reshape(-1, 2) for i in range(4)]
        out["n_runs"] = list(r.n_runs)
        return out

    def check_set_bitmaps(self, cols, words_cap=None, on_device=False, out=None):
        """jh_check_set_bitmaps: the counts plus the four result sets (ok,
        lost, unexpected, recovered) as uint32 bitmaps over [base, base + 32 *
        n_words); bits_to_runs turns one into sorted [lo hi] runs. out: four
        uint32 arrays of words_cap words (e.g. HostBuffers', reused)."""
        h = A.make_history(cols, on_device=on_device)
        r = A.JhSetResult()
        err = C.create_string_buffer(1024)
        p32 = C.POINTER(C.c_uint32)
        base, nw = C.c_int64(), C.c_int64()
        cap = 0 if words_cap is None else int(words_cap)
        if words_cap is None:
            # the element span is bounded by the history's own values (the :add
            # rows' and the reads' elements): size the output from them on the
            # host so the device pass runs once; a device-resident history has
            # no host copy to bound, so it starts small and grows once
            cap = _set_span_words(cols) if not on_device else 1 << 16
        for _ in range(2):
            if out is not None:
                if words_cap is None or len(out) != 4 or any(
                        b.dtype != np.uint32 or len(b) < max(cap, 1) or not b.flags.c_contiguous for b in out):
                    raise ValueError("out: four contiguous uint32 arrays of words_cap words")
                bits = list(out)
            else:
                bits = [np.zeros(max(cap, 1), np.uint32) for _ in range(4)]
            rc = lib().jh_check_set_bitmaps(self._h, C.byref(h), C.byref(r), *[b.ctypes.data_as(p32) for b in bits],
                                            cap, C.byref(base), C.byref(nw), err, len(err))
            _raise(rc, err)
            if nw.value <= cap or words_cap is not None:
                break
            cap = int(nw.value)
        out = {name: getattr(r, name) for name, _ in A.JhSetResult._fields_ if name != "n_runs"}
        out["n_runs"] = list(r.n_runs)
        out["base"], out["n_words"] = base.value, nw.value
        out["bits"] = [b[:min(nw.value, cap)] for b in bits]
        return out

    def check_set_full(self, cols, time, linearizable=False, list_cap=None, on_device=False, read_batch=0):
        """(checker/set-full {:linearizable? linearizable}). `time` is the :time
        column (numpy int64, or a device pointer when on_device); read_batch > 0
        caps the :ok reads per bitmap batch (jh_set_full_opts, tests)."""
        h = A.make_history(cols, on_device=on_device)
        cap = int(cols.n) if list_cap is None else list_cap
        lists = [np.zeros(max(cap, 1), np.int64) for _ in range(3)]
        r = A.JhSetFullResult()
        err = C.create_string_buffer(1024)
        tp = C.cast(C.c_void_p(int(time)), C.POINTER(C.c_int64)) if on_device else A.ptr64(time)
        o = A.JhSetFullOpts(linearizable=int(bool(linearizable)), read_batch=int(read_batch))
        rc = lib().jh_check_set_full_opts(self._h, C.byref(h), tp, C.byref(o), C.byref(r),
                                          *[A.ptr64(x) for x in lists], cap, err, len(err))
        _raise(rc, err)
        out = {name: getattr(r, name) for name, _ in A.JhSetFullResult._fields_}
        out["stable_latencies"] = list(r.stable_latencies)
        out["lost_latencies"] = list(r.lost_latencies)
        out["worst_stale"] = [(w.element, w.stable_latency, w.known_entry, w.last_absent_entry)
                              for w in r.worst_stale[:r.n_worst]]
        for i, nm in enumerate(["lost", "never_read", "stale"]):
            k = min(out[nm + "_count"], cap)
            out[nm] = lists[i][:k]
        return out

    # -- queues --------------------------------------------------------------
    def _queue_out(self, r, pairs, names):
        out = {name: getattr(r, name) for name, _ in A.JhQueueResult._fields_ if name != "n_pairs"}
        out["n_pairs"] = list(r.n_pairs)
        cap = len(pairs[0]) // 2
        for i, nm in enumerate(names):
            out[nm] = pairs[i][:2 * min(r.n_pairs[i], cap)].reshape(-1, 2)
        return out

    def check_total_queue(self, cols, pairs_cap=None, on_device=False):
        h = A.make_history(cols, on_device=on_device)
        cap = (cols.n + (int(cols.n_aux) if on_device else len(cols.aux)) + 1) if pairs_cap is None else pairs_cap
        pairs = [np.zeros(2 * max(cap, 1), np.int64) for _ in range(4)]
        r = A.JhQueueResult()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_total_queue(self._h, C.byref(h), C.byref(r), *[A.ptr64(x) for x in pairs],
                                        cap, err, len(err))
        _raise(rc, err)
        return self._queue_out(r, pairs, ["lost", "unexpected", "duplicated", "recovered"])

    def check_queue(self, cols, pairs_cap=None, on_device=False):
        h = A.make_history(cols, on_device=on_device)
        cap = (cols.n + 1) if pairs_cap is None else pairs_cap
        pairs = [np.zeros(2 * max(cap, 1), np.int64)]
        r = A.JhQueueResult()
        err = C.create_string_buffer(1024)
        rc = lib().jh_check_queue(self._h, C.byref(h), C.byref(r), A.ptr64(pairs[0]), cap, err, len(err))
        _raise(rc, err)
        return self._queue_out(r, pairs, ["final_queue"])


def _set_span_words(cols):
    """Bitmap words covering every element jh_check_set_bitmaps can see: the
    non-nil values of the :add invocations / completions and every read
    element in aux (a superset of the final read's), as jh_set.hip's
    k_set_scan / k_set_range bound [vmin, vmax]."""
    v = np.asarray(cols.value)
    t = np.asarray(cols.type)
    sel = (np.asarray(cols.f) == A.F_ADD) & ((t == A.TYPE_INVOKE) | (t == A.TYPE_OK)) & (v != A.NIL)
    vals = v[sel]
    aux = np.asarray(cols.aux) if cols.aux is not None else np.zeros(0, np.int64)
    lo = min([int(x.min()) for x in (vals, aux) if len(x)], default=0)
    hi = max([int(x.max()) for x in (vals, aux) if len(x)], default=0)
    # (a span over 2^34 elements is refused by the library before any copy)
    return max(1, min(((hi - lo) >> 5) + 2, (1 << 29) + 1))


def bits_to_runs(words, base):
    """Sorted [lo hi] runs of the elements base + i for the set bits i of a
    uint32 bitmap (bit b of word w is element base + 32 w + b)."""
    words = np.ascontiguousarray(words, dtype=np.uint32)
    if words.size == 0:
        return np.zeros((0, 2), np.int64)
    b = np.unpackbits(words.view(np.uint8), bitorder="little").astype(np.int8)
    d = np.diff(np.concatenate(([0], b, [0])))
    lo = np.nonzero(d == 1)[0]
    hi = np.nonzero(d == -1)[0] - 1
    return np.stack([lo + base, hi + base], axis=1).astype(np.int64)


_default = {}


def default_context(device=None):
    """Process-wide context per device (LOCAL_RANK by default)."""
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    with _lock:
        ctx = _default.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _default[device] = ctx
    return ctx
