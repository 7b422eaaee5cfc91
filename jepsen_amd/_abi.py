"""ctypes mirror of include/jh.h (the C ABI of libjh.so).

Kept in one place so the product binding (`_native.py`), the test oracle
wrapper (`oracle/oracle.py`) and the generator wrapper (`synth.py`) agree on
every struct layout.
"""
import ctypes as C

JH_ABI_VERSION = 7

JH_OK, JH_EINVAL, JH_EUNSUPPORTED, JH_EDEVICE, JH_ENOMEM = 0, 1, 2, 3, 4
TYPE_INVOKE, TYPE_OK, TYPE_FAIL, TYPE_INFO = 0, 1, 2, 3
F_READ, F_WRITE, F_CAS, F_ADD = 0, 1, 2, 3
F_ENQUEUE, F_DEQUEUE, F_DRAIN = 4, 5, 6
F_FIRST_INTERNED = 16
NIL = -(1 << 63)

VALID, UNKNOWN, INVALID = 0, 1, 2

CAUSES = {
    0: None,
    1: "budget",
    2: "window",
    3: "double-invoke",
    4: "orphan-completion",
    5: "unsupported-f",
    6: "nil-value",
    7: "overflow",
    8: "states",
    9: "deferred",
}

MAX_WINDOW = 256
DEFAULT_BUDGET = 1 << 20

_p64 = C.POINTER(C.c_int64)


class JhHistory(C.Structure):
    _fields_ = [
        ("n", C.c_int64),
        ("process", _p64),
        ("type", _p64),
        ("f", _p64),
        ("key", _p64),
        ("value", _p64),
        ("value2", _p64),
        ("n_keys", C.c_int64),
        ("aux", _p64),
        ("n_aux", C.c_int64),
        ("on_device", C.c_int32),
        ("reserved", C.c_int32),
    ]


ALGO_COMPETITION, ALGO_WGL, ALGO_LINEAR = 0, 1, 2
ALGORITHMS = {"competition": ALGO_COMPETITION, "wgl": ALGO_WGL, "linear": ALGO_LINEAR}
# jh_lin_opts.flags (test hooks)
LIN_BFS_ONLY, LIN_GEN_JUMP, LIN_INTERN_PER_KEY, LIN_NO_HELPERS, LIN_HELPERS_NOW = 1, 2, 4, 8, 16
LIN_PHASE1_ONLY, LIN_SKIP_PHASE1 = 32, 64
LIN_NO_HANDOVER = 128
LIN_STREAM = 256
LIN_NO_RESUME = 512           # round 5: restart deferred keys instead of continuing them
LIN_EXACT_COUNT = 1024        # round 5: WGL's exact count for every key (the parity tests)
EXPLORED_UNCOUNTED = -3       # a valid key settled without the count pass
LIN_NO_SPEC = 2048            # round 6: no speculative dead-subtree enumerations by idle helpers
LIN_SPEC_FIRST = 4096         # round 6: helpers serve posted spec jobs before taking keys
LIN_HELP_STALL = 8192         # round 6: helpers pick the keys stuck longest (no deeper layer)
LIN_NO_TAKEOVER = 16384       # round 6: forces the takeover off
LIN_TAKEOVER = 32768          # round 6 (opt-in): a helper continues the sequential search's saved state
CAUSE_DEFERRED = 9


class JhLinOpts(C.Structure):
    _fields_ = [("init_value", C.c_int64), ("budget", C.c_int64), ("stream", C.c_int64),
                ("algorithm", C.c_int32), ("flags", C.c_int32),
                ("quick_budget", C.c_int64), ("phase2_budget", C.c_int64),
                ("helpers", C.c_int32), ("helper_late_us", C.c_int32),
                ("xw_waves", C.c_int32), ("p2_waves_per_cu", C.c_int32),
                ("lean_waves", C.c_int32), ("wide_waves", C.c_int32),
                ("handover_min", C.c_int32), ("p1_waves_per_cu", C.c_int32),
                ("bfs_wgs", C.c_int32), ("reserved2", C.c_int32)]       # ABI 7


# every field of jh_key_verdict: the parity tests compare all of them
VERDICT_FIELDS = ("valid", "cause", "fail_entry", "explored", "previous_ok", "last_op", "analyzer")
ANALYZER_WGL, ANALYZER_LINEAR = 0, 1
ANALYZERS = {ANALYZER_WGL: "wgl", ANALYZER_LINEAR: "linear"}


class JhKeyVerdict(C.Structure):
    _fields_ = [("valid", C.c_int32), ("cause", C.c_int32),
                ("fail_entry", C.c_int64), ("explored", C.c_int64),
                ("previous_ok", C.c_int64), ("last_op", C.c_int64),
                ("analyzer", C.c_int32), ("reserved", C.c_int32)]


class JhSummary(C.Structure):
    _fields_ = [("valid", C.c_int64), ("n_invalid", C.c_int64), ("n_unknown", C.c_int64),
                ("first_fail_entry", C.c_int64), ("n_keys", C.c_int64),
                ("explored", C.c_int64), ("memo_probes", C.c_int64),
                ("device_ms", C.c_double), ("dfs_ms", C.c_double),
                ("seq_ms", C.c_double), ("bfs_ms", C.c_double), ("n_deferred", C.c_int64),
                ("deferred_entries", C.c_int64), ("seq_probes", C.c_int64),
                # ABI 4: per-phase accounting
                ("p3_ms", C.c_double), ("wide_ms", C.c_double), ("xw_ms", C.c_double),
                ("p3_probes", C.c_int64), ("wide_probes", C.c_int64), ("xw_probes", C.c_int64),
                ("helper_probes", C.c_int64), ("n_deferred_wide", C.c_int64), ("n_phase3", C.c_int64),
                ("n_phase3_wide", C.c_int64), ("n_xw", C.c_int64), ("lean_entries", C.c_int64),
                ("wide_entries", C.c_int64), ("xw_entries", C.c_int64), ("waves", C.c_int64 * 4),
                # ABI 5: the streaming heavy-key pass
                ("streamed", C.c_int64), ("p3_entries", C.c_int64), ("p2_start_ms", C.c_double),
                ("p1_span_ms", C.c_double),
                # ABI 6: deferred searches resumed by the heavy-key pass
                ("resumed", C.c_int64), ("resume_bytes", C.c_int64),
                # ABI 7: speculative dead-subtree enumerations (round 6)
                ("spec_jobs", C.c_int64), ("spec_dead", C.c_int64), ("spec_merges", C.c_int64),
                ("spec_nodes", C.c_int64), ("takeovers", C.c_int64)]


class JhLinConfig(C.Structure):
    _fields_ = [("key", C.c_int64), ("model_value", C.c_int64), ("n_linearized", C.c_int32),
                ("n_pending", C.c_int32), ("rows_off", C.c_int64),
                ("last_row", C.c_int64)]            # ABI 6: the :ok completion that is :last-op


CONFIGS_PER_KEY = 10          # checker.clj:146-158: (take 10 ...) of :configs and :final-paths


class JhSetResult(C.Structure):
    _fields_ = [("valid", C.c_int32), ("cause", C.c_int32),
                ("attempt_count", C.c_int64), ("acknowledged_count", C.c_int64),
                ("ok_count", C.c_int64), ("lost_count", C.c_int64),
                ("recovered_count", C.c_int64), ("unexpected_count", C.c_int64),
                ("first_fail_entry", C.c_int64), ("final_read_entry", C.c_int64),
                ("n_runs", C.c_int64 * 4)]


SF_QUANTILES = 5
SF_WORST = 8
SF_POINTS = (0, 0.5, 0.95, 0.99, 1)       # checker.clj:412


class JhSetFullElem(C.Structure):
    _fields_ = [("element", C.c_int64), ("stable_latency", C.c_int64),
                ("known_entry", C.c_int64), ("last_absent_entry", C.c_int64)]


class JhSetFullResult(C.Structure):
    _fields_ = [("valid", C.c_int32), ("cause", C.c_int32),
                ("attempt_count", C.c_int64), ("stable_count", C.c_int64),
                ("lost_count", C.c_int64), ("never_read_count", C.c_int64),
                ("stale_count", C.c_int64),
                ("has_stable_latencies", C.c_int32), ("has_lost_latencies", C.c_int32),
                ("stable_latencies", C.c_int64 * SF_QUANTILES),
                ("lost_latencies", C.c_int64 * SF_QUANTILES),
                ("n_worst", C.c_int64), ("worst_stale", JhSetFullElem * SF_WORST),
                ("n_reads", C.c_int64), ("read_elements", C.c_int64),
                ("device_ms", C.c_double)]


class JhSetFullOpts(C.Structure):
    _fields_ = [("linearizable", C.c_int32), ("pad", C.c_int32), ("read_batch", C.c_int64),
                ("reserved", C.c_int64 * 4)]


class JhIngestOpts(C.Structure):
    """include/jh_io.h jh_ingest_opts."""
    _fields_ = [("threads", C.c_int32), ("debug", C.c_int32), ("min_chunk", C.c_int64),
                ("reserved", C.c_int64 * 4)]


class JhQueueResult(C.Structure):
    _fields_ = [("valid", C.c_int32), ("cause", C.c_int32),
                ("attempt_count", C.c_int64), ("acknowledged_count", C.c_int64),
                ("ok_count", C.c_int64), ("unexpected_count", C.c_int64),
                ("duplicated_count", C.c_int64), ("lost_count", C.c_int64),
                ("recovered_count", C.c_int64), ("n_pairs", C.c_int64 * 4),
                ("fail_entry", C.c_int64), ("fail_value", C.c_int64), ("device_ms", C.c_double)]


# numpy structured dtype with the same layout as jh_key_verdict
try:
    import numpy as _np
    VERDICT_DTYPE = _np.dtype([("valid", _np.int32), ("cause", _np.int32),
                               ("fail_entry", _np.int64), ("explored", _np.int64),
                               ("previous_ok", _np.int64), ("last_op", _np.int64),
                               ("analyzer", _np.int32), ("reserved", _np.int32)])
except Exception:  # pragma: no cover
    VERDICT_DTYPE = None


def ptr64(a):
    """int64* for a C-contiguous numpy int64 array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(_p64)


def make_history(cols, on_device=False):
    """Build a JhHistory from an object with numpy (or device-pointer) columns.

    `cols` must have attributes n, process, type, f, key, value, value2,
    n_keys, aux (may be None)."""
    h = JhHistory()
    h.n = int(cols.n)
    if on_device:
        def dp(x):
            return C.cast(C.c_void_p(int(x)), _p64) if x else None
        h.process, h.type, h.f = dp(cols.process), dp(cols.type), dp(cols.f)
        h.key, h.value, h.value2 = dp(cols.key), dp(cols.value), dp(cols.value2)
        h.aux = dp(getattr(cols, "aux", 0))
        h.on_device = 1
    else:
        h.process, h.type, h.f = ptr64(cols.process), ptr64(cols.type), ptr64(cols.f)
        h.key, h.value, h.value2 = ptr64(cols.key), ptr64(cols.value), ptr64(cols.value2)
        h.aux = ptr64(cols.aux) if getattr(cols, "aux", None) is not None else None
        h.on_device = 0
    h.n_keys = int(cols.n_keys)
    aux = getattr(cols, "aux", None)
    h.n_aux = int(len(aux)) if (aux is not None and not on_device) else int(getattr(cols, "n_aux", 0))
    return h
