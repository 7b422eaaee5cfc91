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
from .model import CASRegister, Mutex, Register, UnorderedQueue, is_inconsistent, to_device_ops

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
    "states": "more distinct register values in one key than the device state encoding holds",
}


class Analysis(dict):
    """A result map of checker/linearizable, plus the ABI's per-key side
    channel as attributes -- not map keys. checker.clj:156-158 returns
    knossos' analysis with :final-paths and :configs assoc'ed on, and the
    reference's printed analysis (doc/tutorial/04-checker.md:126-138) has no
    :explored or failing-row key; jh_key_verdict's `explored` (WGL's cache
    size, the count the parity tests compare with the oracle) and
    `fail_entry` (the failing op's row) ride along here, where the JVM shim
    keeps them out of the Clojure map as well."""
    __slots__ = ("explored", "fail_entry")

    def __init__(self, m, explored=-1, fail_entry=-1):
        super().__init__(m)
        self.explored = explored
        self.fail_entry = fail_entry


def lin_result(valid, cause, fail_entry, explored, cols=None, previous_ok=-1, last_op=-1, analyzer=A.ANALYZER_WGL,
               ops=None):
    """Per-history result map of checker/linearizable (checker.clj:139-158):
    the analysis with :configs and :final-paths assoc'ed on (empty until
    add_configs fills them) and :analyzer, the analysis that decided the key
    (jh_key_verdict.analyzer: :wgl, or :linear under {:algorithm :linear}).
    An invalid result carries :op (the ok completion no configuration gets
    past) and, from the search frontier, :previous-ok and :last-op (include/jh.h;
    knossos is not vendored, so their exact knossos definitions are parity
    unpinned). ops: the history's op maps, when the caller has them (op maps
    are then the caller's own, :time and all)."""
    c = A.CAUSES.get(int(cause))
    an = A.ANALYZERS.get(int(analyzer), "wgl")
    side = dict(explored=int(explored), fail_entry=int(fail_entry))
    if valid == A.VALID:
        return Analysis({"valid?": True, "configs": [], "analyzer": an, "final-paths": []}, **side)
    if valid == A.INVALID:
        r = {"valid?": False}
        if cols is not None and 0 <= fail_entry < cols.n:
            r["op"] = op_at(cols, ops, int(fail_entry))
        if cols is not None:
            r["previous-ok"] = op_at(cols, ops, int(previous_ok)) if 0 <= previous_ok < cols.n else None
            r["last-op"] = op_at(cols, ops, int(last_op)) if 0 <= last_op < cols.n else None
        r.update({"configs": [], "analyzer": an, "final-paths": []})
        return Analysis(r, **side)
    if c == "budget":
        return Analysis({"valid?": UNKNOWN, "cause": "budget", "configs": [], "analyzer": an, "final-paths": []},
                        **side)
    return Analysis({"valid?": UNKNOWN, "error": CAUSE_ERRORS.get(c, c), "cause": c}, **side)


def op_at(cols, ops, row):
    """The op map at a history row: the caller's own map when it passed op
    maps (knossos hands its analysis the history's maps; their :index is the
    full history's, core.clj:441), else decoded from the columns. An
    independent tuple value is unwrapped, as subhistory does
    (independent.clj:234-245)."""
    if ops is not None and 0 <= row < len(ops):
        op = dict(ops[row])
        op.setdefault("index", row)
    else:
        op = H.decode_op(cols, int(row))
    return _unwrap(op)


class Linearizable(Checker):
    """checker.clj:127-158 with {:model (cas-register v)}. :algorithm :wgl and
    the default (competition) report the WGL analysis; :linear runs the
    JIT-linearization analysis (the reachable configuration set) on every
    key it can hold and WGL on the rest -- each key's :analyzer says which.
    Both are complete decision procedures: :valid? is the same."""

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
        ops = None
        if not isinstance(history, H.Columns):
            ops = list(history)
            history = to_device_ops(self.model, ops)
        cols = _cols(history, keyed=False)
        init = _init_state(self.model, cols)
        r = _ctx().check_cas_full(cols, init=init, budget=self.budget, algorithm=_algorithm(self.algorithm),
                                  exact_count=False)
        out = lin_result(r["valid"], r["cause"], r["fail_entry"], r["explored"], cols,
                         r["previous_ok"], r["last_op"], r["analyzer"], ops=ops)
        if wants_configs(r["valid"], r["analyzer"]):
            cf = _ctx().lin_configs(cols, [0], init=init, budget=self.budget)
            add_configs(out, cf[0], cols, self.model, ops=ops)
            from .report import maybe_render
            maybe_render(test, opts, cols, out)
        return out


def wants_configs(valid, analyzer):
    """Which analyses carry :configs (checker.clj:156-158 keeps (take 10 ...)):
    an invalid one's frontier, and a valid :linear one's final configurations
    (doc/tutorial/04-checker.md:126-138 prints one). A valid WGL analysis has
    none."""
    return int(valid) == A.INVALID or (int(valid) == A.VALID and int(analyzer) == A.ANALYZER_LINEAR)


def add_configs(result, configs, cols, model=None, ops=None):
    """:configs and :final-paths (checker.clj:146-158 keeps (take 10 ...) of
    each), from jh_lin_configs: an invalid key's frontier -- the
    configurations at the last layer any search reaches -- or a valid :linear
    key's final configurations, first 10 in the canonical order (include/jh.h).

    A configuration is shaped as knossos' analysis prints one
    (doc/tutorial/04-checker.md:128-135): the model; :last-op, the :ok
    completion of the last op linearized, with its own :index (jh_lin_config
    .last_row); :pending, the ops invoked and not linearized, in call order.
    A final path (invalid keys only) starts at the configuration
    ({:op last-op :model model}), linearizes the pending ops that step
    consistently, in call order, each with the model after it, and ends in
    the failing :op, inconsistent from every frontier model (a model it could
    step from would have a successor past the op's completion) -- one path
    per configuration. knossos is not vendored: the path choice is this
    library's, parity unpinned."""
    if configs is None:
        return result
    cf = []
    for v, lin, pend, last_row in configs:
        val = None if v == A.NIL else int(v)
        if val is not None and cols.values_interned and 0 <= val < len(cols.value_table):
            val = cols.value_table[val]          # interned history: the state is a value-table id
        m = _model_of(model, val)
        cf.append({"model": _model_map(m),
                   "last-op": op_at(cols, ops, last_row) if last_row >= 0 else None,
                   "pending": [_completed_op(cols, x, ops) for x in pend],
                   "_m": m})
    op = result.get("op")
    paths = []
    if result.get("valid?") is False:
        for c in cf[:A.CONFIGS_PER_KEY]:
            m = c["_m"]
            path = [{"op": c["last-op"], "model": _model_map(m)}]
            for p in c["pending"]:
                r = _step(m, p)
                if r is None or is_inconsistent(r):
                    continue
                m = r
                path.append({"op": p, "model": _model_map(m)})
            if op is not None:
                r = _step(m, op)
                path.append({"op": op, "model": ({"inconsistent": r.msg} if is_inconsistent(r) else
                                                 {"error": "no step"} if r is None else _model_map(r))})
            paths.append(path)
    for c in cf:
        del c["_m"]
    result["configs"] = cf[:A.CONFIGS_PER_KEY]
    result["final-paths"] = paths
    return result


def _next_same_process(cols):
    """For every row, the next row of the same process (-1 if none): one
    stable sort per history, cached on the columns (a scan of the
    whole column per op cost more than the device check on big histories)."""
    nxt = getattr(cols, "_next_same_proc", None)
    if nxt is None:
        order = np.argsort(cols.process, kind="stable")
        nxt = np.full(cols.n, -1, np.int64)
        same = cols.process[order[1:]] == cols.process[order[:-1]]
        nxt[order[:-1][same]] = order[1:][same]
        cols._next_same_proc = nxt
    return nxt


def _completed_op(cols, row, ops=None):
    """The invocation at `row` as knossos.history/complete leaves it [K]
    (cassandra/src/cassandra/checker.clj:29-31): an :ok completion fills a
    nil :value -- the next row of the same process completes it."""
    op = op_at(cols, ops, int(row))
    if op.get("value") is None:
        p = int(cols.process[row])
        if p >= 0:
            c = int(_next_same_process(cols)[row])
            if c >= 0 and int(cols.type[c]) == A.TYPE_OK:
                op = dict(op, value=op_at(cols, ops, c).get("value"))
    return op


def _unwrap(op):
    v = op.get("value")
    if H.is_tuple(v):                                   # an independent tuple
        op = dict(op, value=v.val)
    return op


def _model_of(model, value):
    """The model object for a configuration's interned state value."""
    if isinstance(model, Mutex):
        return Mutex(bool(value))
    if isinstance(model, Register):
        return Register(value)
    return CASRegister(value)


def _model_map(m):
    if isinstance(m, Mutex):
        return {"locked": m.locked}
    return {"value": getattr(m, "value", None)}


def _step(m, op):
    """knossos.model/step of model m on a history op map (mutex ops arrive as
    the cas they were searched as, model.to_device_ops); None if no clause."""
    op = _unwrap(op)
    if isinstance(m, Mutex):
        cas = op.get("value")
        if op.get("f") == "cas":
            op = dict(op, f="acquire" if list(cas or []) == [0, 1] else "release")
    try:
        return m.step(op)
    except (ValueError, TypeError):
        return None


def _algorithm(a):
    """checker.clj:141-145: (case (:algorithm opts) :linear ... :wgl ... competition)."""
    a = (a or "competition")
    a = a.lstrip(":") if isinstance(a, str) else a
    return A.ALGORITHMS.get(a, A.ALGO_COMPETITION)


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
        from ._native import bits_to_runs
        cols = _cols(history, keyed=False)
        r = _ctx().check_set_bitmaps(cols)
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
            out[nm] = _runs_str(bits_to_runs(r["bits"][i], r["base"]).tolist())
        return out


def set():  # noqa: A001 - the reference's name (checker.clj:182)
    return SetChecker()


class SetFull(Checker):
    """(checker/set-full {:linearizable? b}), checker.clj:236-534.

    Same result map as the reference: per-element outcomes counted on the
    device (jh_check_set_full); :worst-stale entries carry the :known and
    :last-absent op maps of the history."""

    def __init__(self, checker_opts=None):
        self.opts = dict(checker_opts or {"linearizable?": False})

    def check(self, test, history, opts):
        ops = None if isinstance(history, H.Columns) else list(history)
        cols = _cols(ops if ops is not None else history, keyed=False)
        if not cols.ints_only:
            raise TypeError("set-full elements must be integers on the device path")
        if ops is not None:
            time = np.asarray([int(o.get("time", 0) or 0) for o in ops], np.int64)
        else:
            time = getattr(cols, "time", None)
            if time is None:
                raise ValueError("set-full needs the :time of every op")
        if len(time) == 0:
            time = np.zeros(1, np.int64)
        r = _ctx().check_set_full(cols, time, linearizable=bool(self.opts.get("linearizable?")))
        return set_full_result(r, ops if ops is not None else cols, time)


def set_full_result(r, ops, time=None):
    """The (checker/set-full) result map from a jh_check_set_full result."""
    def op_at(i):
        if i is None or i < 0:
            return None
        if isinstance(ops, H.Columns):
            o = H.decode_op(ops, int(i))
            o["index"] = int(i)
            if time is not None:
                o["time"] = int(time[i])
            return o
        return ops[int(i)]

    valid = {A.VALID: True, A.INVALID: False}.get(r["valid"], UNKNOWN)
    worst = [{"element": int(e), "outcome": "stable", "stable-latency": int(lat),
              "lost-latency": None, "known": op_at(k), "last-absent": op_at(la)}
             for e, lat, k, la in r["worst_stale"]]
    m = {"valid?": valid,
         "attempt-count": int(r["attempt_count"]),
         "stable-count": int(r["stable_count"]),
         "lost-count": int(r["lost_count"]),
         "lost": [int(x) for x in r["lost"]],
         "never-read-count": int(r["never_read_count"]),
         "never-read": [int(x) for x in r["never_read"]],
         "stale-count": int(r["stale_count"]),
         "stale": [int(x) for x in r["stale"]],
         "worst-stale": worst}
    if r["has_stable_latencies"]:
        m["stable-latencies"] = dict(zip(A.SF_POINTS, (int(x) for x in r["stable_latencies"])))
    if r["has_lost_latencies"]:
        m["lost-latencies"] = dict(zip(A.SF_POINTS, (int(x) for x in r["lost_latencies"])))
    # (frequencies v) counts are >= 1, so `(< v 1)` never holds (checker.clj:505-510)
    m["duplicated-count"] = 0
    m["duplicated"] = {}
    return m


def set_full(checker_opts=None):
    return SetFull(checker_opts)


def _unscalar(cols, x):
    x = int(x)
    if x == A.NIL:
        return None
    return cols.value_table[x] if cols.values_interned else x


def _multiset(cols, pairs):
    """(value, multiplicity) pairs -> collections.Counter (a multiset)."""
    from collections import Counter
    return Counter({_unscalar(cols, v): int(c) for v, c in pairs})


class Queue(Checker):
    """(checker/queue model), checker.clj:160-180, for knossos'
    unordered-queue model (jh_check_queue)."""

    def __init__(self, model):
        self.model = model

    def check(self, test, history, opts):
        ops = None if isinstance(history, H.Columns) else list(history)
        if self.model is None:
            if ops is not None and not ops:
                return {"valid?": True, "final-queue": None}
            raise TypeError("(queue nil): model/step on nil")
        if not isinstance(self.model, UnorderedQueue) or self.model.pending:
            raise TypeError("the device queue checker takes an empty (model/unordered-queue)")
        cols = _cols(ops if ops is not None else history, keyed=False)
        r = _ctx().check_queue(cols)
        if r["valid"] == A.INVALID:
            return {"valid?": False, "error": "can't dequeue %s" % (_unscalar(cols, r["fail_value"]),),
                    "fail-entry": int(r["fail_entry"])}
        return {"valid?": True, "final-queue": _multiset(cols, r["final_queue"])}


def queue(model):
    return Queue(model)


class TotalQueue(Checker):
    """(checker/total-queue), checker.clj:536-628 (jh_check_total_queue)."""

    def check(self, test, history, opts):
        cols = _cols(history, keyed=False)
        r = _ctx().check_total_queue(cols)
        out = {"valid?": bool(r["valid"] == A.VALID)}
        for k in ("attempt", "acknowledged", "ok", "unexpected", "duplicated", "lost", "recovered"):
            out[k + "-count"] = int(r[k + "_count"])
        for k in ("lost", "unexpected", "duplicated", "recovered"):
            out[k] = _multiset(cols, r[k])
        return out


def total_queue():
    return TotalQueue()
