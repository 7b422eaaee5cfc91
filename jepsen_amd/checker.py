"""jepsen.checker on MI355X: the Checker protocol, its combinators, and the
device-backed linearizable / counter / set checkers.

Mirrors jepsen/src/jepsen/checker.clj (names, argument meaning, result maps,
error behaviour). Result maps use the reference's keyword names as strings
("valid?", "reads", "attempt-count", ...); :unknown is the string "unknown".
"""
import builtins
import traceback

import numpy as np

from . import _abi as A
from . import history as H
from .model import CASRegister, Mutex, Register, to_device_ops

UNKNOWN = "unknown"

# checker.clj:26-31
VALID_PRIORITIES = {True: 0, False: 1, UNKNOWN: 0.5}


def _prio(v):
    for k, p in VALID_PRIORITIES.items():
        if v is k or (v == k and type(v) is type(k)):
            return p
    raise ValueError(f"{v!r} is not a known valid? value")


def merge_valid(valids):
    """checker.clj:33-47: the highest-priority :valid? value, starting from true."""
    out = True
    for v in valids:
        if _prio(out) < _prio(v):
            out = v
    return out


class Checker:
    """checker.clj:49-69 (defprotocol Checker (check [checker test history opts]))."""

    def check(self, test, history, opts):
        raise NotImplementedError


def check(checker, test, history, opts=None):
    return checker.check(test, history, opts or {})


class _Fn(Checker):
    def __init__(self, fn):
        self.fn = fn

    def check(self, test, history, opts):
        return self.fn(test, history, opts)


def noop():
    """checker.clj:71-75"""
    return _Fn(lambda t, h, o: None)


def unbridled_optimism():
    """checker.clj:121-125"""
    return _Fn(lambda t, h, o: {"valid?": True})


def check_safe(checker, test, history, opts=None):
    """checker.clj:77-88: exceptions become {:valid? :unknown :error trace}."""
    try:
        return checker.check(test, history, opts or {})
    except Exception:
        return {"valid?": UNKNOWN, "error": traceback.format_exc()}


class Compose(Checker):
    """checker.clj:90-102 (the reference runs the members under pmap)."""

    def __init__(self, checker_map):
        self.checker_map = dict(checker_map)

    def check(self, test, history, opts):
        results = {k: check_safe(c, test, history, opts) for k, c in self.checker_map.items()}
        results["valid?"] = merge_valid(r.get("valid?") if isinstance(r, dict) else None
                                        for r in results.values())
        return results


def compose(checker_map):
    return Compose(checker_map)


def concurrency_limit(limit, checker):
    """checker.clj:104-119 (a fair semaphore around check)."""
    import threading
    sem = threading.BoundedSemaphore(limit)

    def run(t, h, o):
        with sem:
            return checker.check(t, h, o)
    return _Fn(run)


# ---------------------------------------------------------------------------
def integer_interval_set_str(s):
    """util.clj:536-575: "#{1..3 5 7..9}"."""
    if any(x is None for x in s):
        return "#{" + " ".join(str(x) for x in s) + "}"
    xs = sorted(builtins.set(int(x) for x in s))
    return _runs_str(_to_runs(xs))


def _to_runs(xs):
    runs = []
    for x in xs:
        if runs and runs[-1][1] + 1 == x:
            runs[-1][1] = x
        else:
            runs.append([x, x])
    return runs


def _runs_str(runs):
    parts = [str(a) if a == b else f"{a}..{b}" for a, b in runs]
    return "#{" + " ".join(parts) + "}"


def _cols(history, keyed=False):
    if isinstance(history, H.Columns):
        return history
    return H.encode(list(history), keyed=keyed)


def _ctx():
    from . import _native
    return _native.default_context()


def _init_state(model, cols):
    v = model.value
    if v is None:
        return A.NIL
    if cols.values_interned:
        for i, x in enumerate(cols.value_table):
            if x == v and type(x) is type(v):
                return i
        return len(cols.value_table)
    return int(v)


CAUSE_ERRORS = {
    "double-invoke": "knossos.history/complete: process already running, yet attempted to invoke concurrently",
    "orphan-completion": "knossos.history/complete: completion without an outstanding invocation",
    "unsupported-f": "IllegalArgumentException: the cas-register model has no step for this :f",
    "window": "more concurrent operations than the device search window supports",
}


def lin_result(valid, cause, fail_entry, explored, cols=None):
    """Per-history result map of checker/linearizable (checker.clj:139-158)."""
    c = A.CAUSES.get(int(cause))
    if valid == A.VALID:
        return {"valid?": True, "analyzer": "wgl", "explored": int(explored)}
    if valid == A.INVALID:
        r = {"valid?": False, "analyzer": "wgl", "explored": int(explored),
             "fail-entry": int(fail_entry)}
        if cols is not None and 0 <= fail_entry < cols.n:
            r["op"] = H.decode_op(cols, int(fail_entry))
        return r
    if c == "budget":
        return {"valid?": UNKNOWN, "analyzer": "wgl", "cause": "budget", "explored": int(explored)}
    return {"valid?": UNKNOWN, "error": CAUSE_ERRORS.get(c, c), "cause": c}


class Linearizable(Checker):
    """checker.clj:127-158 with {:model (cas-register v)}; every :algorithm
    (:linear, :wgl, competition) decides the same :valid?."""

    def __init__(self, opts):
        model = opts.get("model")
        assert model is not None, ("The linearizable checker requires a model. It received: "
                                   f"{model} instead.")
        self.model = model
        self.algorithm = opts.get("algorithm")
        self.budget = opts.get("budget")

    def supported(self):
        return isinstance(self.model, (CASRegister, Register, Mutex))

    def check(self, test, history, opts):
        if not self.supported():
            raise NotImplementedError(f"model {self.model!r} has no device implementation")
        if not isinstance(history, H.Columns):
            history = to_device_ops(self.model, list(history))
        cols = _cols(history, keyed=False)
        v, c, fe, ex = _ctx().check_cas(cols, init=_init_state(self.model, cols), budget=self.budget)
        return lin_result(v, c, fe, ex, cols)


def linearizable(opts):
    return Linearizable(opts)


class Counter(Checker):
    """checker.clj:679-734."""

    def check(self, test, history, opts):
        cols = _cols(history, keyed=False)
        if not cols.ints_only:
            raise TypeError("counter values must be integers")
        r = _ctx().check_counter(cols)
        if r["valid"] == A.UNKNOWN:
            raise ArithmeticError(f"counter check failed: {A.CAUSES.get(r['cause'])}")
        reads = r["reads"]
        bad = ~((reads[:, 0] <= reads[:, 1]) & (reads[:, 1] <= reads[:, 2])) if len(reads) else np.zeros(0, bool)
        return {"valid?": bool(r["valid"] == A.VALID),
                "reads": reads.tolist(),
                "errors": reads[bad].tolist()}


def counter():
    return Counter()


class SetChecker(Checker):
    """checker.clj:182-233."""

    def check(self, test, history, opts):
        cols = _cols(history, keyed=False)
        r = _ctx().check_set(cols)
        if r["valid"] == A.UNKNOWN:
            return {"valid?": UNKNOWN, "error": "Set was never read"}
        names = ["ok", "lost", "unexpected", "recovered"]
        out = {"valid?": bool(r["valid"] == A.VALID),
               "attempt-count": int(r["attempt_count"]),
               "acknowledged-count": int(r["acknowledged_count"]),
               "ok-count": int(r["ok_count"]),
               "lost-count": int(r["lost_count"]),
               "recovered-count": int(r["recovered_count"]),
               "unexpected-count": int(r["unexpected_count"])}
        for i, nm in enumerate(names):
            out[nm] = _runs_str(r["runs"][i].tolist())
        return out


def set():  # noqa: A001 - the reference's name (checker.clj:182)
    return SetChecker()
