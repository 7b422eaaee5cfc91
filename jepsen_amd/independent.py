"""jepsen.independent on MI355X (jepsen/src/jepsen/independent.clj).

`checker(inner)` lifts a checker over [k v] tuples. When the inner checker
is (or composes) a cas-register `linearizable`, the whole history is encoded
once and ALL keys are checked by one libjh call (splitter + per-key WGL on
the GPU); any other composed checkers still run per key on their own.
"""
from . import _abi as A
from . import history as H
from .checker import (Checker, Compose, Linearizable, _algorithm, add_configs, check_safe, lin_result, merge_valid,
                      wants_configs, _init_state, _ctx)
from .model import to_device_ops

DIR = "independent"
tuple_ = H.tuple_
is_tuple = H.is_tuple


def history_keys(history):
    """independent.clj:222-232 (in first-appearance order)."""
    seen = {}
    for op in history:
        v = op.get("value")
        if is_tuple(v) and v.key not in seen:
            seen[v.key] = True
    return list(seen)


def subhistory(k, history):
    """independent.clj:234-245: un-keyed ops plus the ops of key k, unwrapped."""
    out = []
    for op in history:
        v = op.get("value")
        if not is_tuple(v):
            out.append(op)
        elif v.key == k:
            o = dict(op)
            o["value"] = v.val
            out.append(o)
    return out


def subhistories(history, keys=None):
    """{k: (subhistory k history)} for every key at once, in ONE pass over the
    history (O(N + K*U) for U un-keyed ops) instead of the reference's one
    O(N) scan per key (independent.clj:234-245, called per key at :266-275).
    Each list is exactly what `subhistory` returns for its key: the un-keyed
    ops and the key's ops unwrapped, in history order."""
    if keys is None:
        keys = history_keys(history)
    out = {k: [] for k in keys}
    for op in history:
        v = op.get("value")
        if not is_tuple(v):
            for lst in out.values():
                lst.append(op)
        else:
            lst = out.get(v.key)
            if lst is not None:
                o = dict(op)
                o["value"] = v.val
                lst.append(o)
    return out


def subhistories_indexed(history, key_off, rows, key_ids):
    """The same lists as `subhistories`, built from libjh's per-key row index
    (jh_key_index: the device's stable key partition). Key k's subhistory is
    its rows merged with the un-keyed rows, both already in history order, so
    building all of them is one O(N + K*U) pass with no scan per key.
    key_ids: {key: dense key id of the encoding}."""
    import numpy as np
    unkeyed = rows[key_off[-1]:]
    out = {}
    for key, kid in key_ids.items():
        mine = rows[key_off[kid]:key_off[kid + 1]]
        merged = np.sort(np.concatenate([mine, unkeyed])) if len(unkeyed) else mine
        lst = []
        for r in merged.tolist():
            op = history[r]
            v = op.get("value")
            if is_tuple(v):
                op = dict(op)
                op["value"] = v.val
            lst.append(op)
        out[key] = lst
    return out


def _lin_member(inner):
    if isinstance(inner, Linearizable) and inner.supported():
        return None, inner
    if isinstance(inner, Compose):
        for name, c in inner.checker_map.items():
            if isinstance(c, Linearizable) and c.supported():
                return name, c
    return None, None


class IndependentChecker(Checker):
    """independent.clj:247-298."""

    def __init__(self, inner):
        self.inner = inner

    def _results_map(self, results):
        failures = [k for k, r in results.items() if not r.get("valid?")]
        return {"valid?": merge_valid(r.get("valid?") for r in results.values()),
                "results": results,
                "failures": failures}

    def check(self, test, history, opts):
        history = list(history)
        name, lin = _lin_member(self.inner)
        if lin is not None:
            try:
                dev_history = to_device_ops(lin.model, history)
            except ValueError:
                dev_history = None        # an op the model has no clause for: per key below
        if lin is not None and dev_history is not None:
            cols = H.encode(dev_history, keyed=True)
            unkeyed_client = any(int(p) >= 0 and int(k) < 0 for p, k in zip(cols.process, cols.key))
            if cols.n_keys and not unkeyed_client:
                verdicts, _ = _ctx().check_cas_independent(
                    cols, init=_init_state(lin.model, cols), budget=lin.budget,
                    algorithm=_algorithm(lin.algorithm), exact_count=False)
                lin_res = {}
                for kid, key in enumerate(cols.keys):
                    v = verdicts[kid]
                    if int(v["explored"]) == -1:      # a key in no tuple: no :results entry
                        continue
                    lin_res[key] = lin_result(int(v["valid"]), int(v["cause"]), int(v["fail_entry"]),
                                              int(v["explored"]), cols, int(v["previous_ok"]),
                                              int(v["last_op"]), int(v["analyzer"]), ops=history)
                want = [kid for kid, key in enumerate(cols.keys)
                        if key in lin_res and wants_configs(verdicts[kid]["valid"], verdicts[kid]["analyzer"])]
                if want:
                    # every invalid key's frontier and every valid :linear key's
                    # final configurations, one device call (jh_lin_configs)
                    cf = _ctx().lin_configs(cols, want, init=_init_state(lin.model, cols), budget=lin.budget)
                    from .report import maybe_render
                    for kid in want:
                        add_configs(lin_res[cols.keys[kid]], cf[kid], cols, lin.model, ops=history)
                        maybe_render(test, {"subdirectory": [DIR, cols.keys[kid]]}, cols, lin_res[cols.keys[kid]])
                if name is None:
                    return self._results_map(lin_res)
                results = {}
                ctx = _ctx()
                key_off, rows = ctx.key_index(cols)
                kid_of = {key: kid for kid, key in enumerate(cols.keys) if key in lin_res}
                subs = subhistories_indexed(history, key_off, rows, kid_of)
                for key, lr in lin_res.items():
                    sub = subs[key]
                    r = {}
                    for nm, c in self.inner.checker_map.items():
                        r[nm] = lr if nm == name else check_safe(
                            c, test, sub, {"subdirectory": [DIR, key], "history-key": key})
                    r["valid?"] = merge_valid(x.get("valid?") if isinstance(x, dict) else None
                                              for x in r.values())
                    results[key] = r
                return self._results_map(results)
        # generic path: every key through the inner checker (per-key device
        # calls for a linearizable inner)
        results = {}
        for key, sub in subhistories(history).items():
            results[key] = check_safe(self.inner, test, sub,
                                      {"subdirectory": [DIR, key], "history-key": key})
        return self._results_map(results)


def checker(inner):
    return IndependentChecker(inner)
