"""knossos.model/register and knossos.model/mutex on the cas-register search
(jepsen_amd/model.py `to_device_ops`). No GPU: the translation is checked
against a brute-force linearizability search that uses the models' own
`step` (the spec), through the CPU oracle on the translated history.
knossos is not vendored, so both models' semantics are parity unpinned
beyond that restatement."""
import itertools
import random

import pytest

from jepsen_amd import _abi as A
from jepsen_amd import history as H
from jepsen_amd import model as M
from oracle import oracle


def _brute(model, history):
    """Herlihy-Wing from the definition, with `model.step`: some order of all
    :ok ops and any subset of :info ops, respecting real time, is legal."""
    calls, open_ = [], {}
    for i, op in enumerate(history):
        p = op["process"]
        if op["type"] == "invoke":
            open_[p] = len(calls)
            calls.append({"op": op, "inv": i, "ret": None, "kind": None})
        else:
            c = calls[open_.pop(p)]
            # a crashed (:info) op never returned: it stays concurrent with
            # everything after its invocation
            c["ret"], c["kind"] = (None if op["type"] == "info" else i), op["type"]
            if op["type"] == "ok" and c["op"].get("value") is None:
                c["op"] = dict(c["op"], value=op.get("value"))
    for c in calls:
        if c["kind"] is None:
            c["kind"] = "info"
    ok = [c for c in calls if c["kind"] == "ok"]
    crashed = [c for c in calls if c["kind"] == "info"]
    for r in range(len(crashed) + 1):
        for extra in itertools.combinations(crashed, r):
            chosen = ok + list(extra)
            for perm in itertools.permutations(chosen):
                good, m = True, model
                for a, b in itertools.combinations(range(len(perm)), 2):
                    x, y = perm[a], perm[b]
                    if y["ret"] is not None and y["ret"] < x["inv"]:
                        good = False
                        break
                if not good:
                    continue
                for c in perm:
                    m = m.step(c["op"])
                    if M.is_inconsistent(m):
                        break
                else:
                    return True
    return False


def _random_mutex_history(rng, n_procs=3, n_ops=5):
    h, busy, done = [], {}, 0
    while done < n_ops or busy:
        p = rng.randrange(n_procs)
        if p in busy:
            f = busy.pop(p)
            t = rng.choice(["ok", "ok", "ok", "fail", "info"])
            h.append({"process": p, "type": t, "f": f, "value": None})
        elif done < n_ops:
            f = rng.choice(["acquire", "release"])
            busy[p] = f
            h.append({"process": p, "type": "invoke", "f": f, "value": None})
            done += 1
    # a crashed process never completes again: drop ops after its :info
    out, dead = [], set()
    for op in h:
        if op["process"] in dead:
            continue
        out.append(op)
        if op["type"] == "info":
            dead.add(op["process"])
    return out


def test_mutex_translation_matches_brute_force(built):
    rng = random.Random(7)
    seen = {A.VALID: 0, A.INVALID: 0}
    for _ in range(300):
        h = _random_mutex_history(rng)
        # :fail ops never took effect: the brute force drops them, as
        # knossos.history/complete marks them :fails?
        failed = set()
        inv_at = {}
        for i, op in enumerate(h):
            if op["type"] == "invoke":
                inv_at[op["process"]] = i
            elif op["type"] == "fail":
                failed.add(inv_at[op["process"]])
                failed.add(i)
        hf = [op for i, op in enumerate(h) if i not in failed]
        exp = _brute(M.mutex(), hf)
        cols = H.encode(M.to_device_ops(M.mutex(), h), keyed=False)
        got = oracle.check_cas(cols, init=0)[0]
        assert got == (A.VALID if exp else A.INVALID), h
        seen[got] += 1
    assert seen[A.VALID] > 20 and seen[A.INVALID] > 20


def test_mutex_known_cases(built):
    def run(h):
        cols = H.encode(M.to_device_ops(M.mutex(), h), keyed=False)
        return oracle.check_cas(cols, init=0)[0]
    acq = lambda p, t: {"process": p, "type": t, "f": "acquire", "value": None}
    rel = lambda p, t: {"process": p, "type": t, "f": "release", "value": None}
    assert run([acq(0, "invoke"), acq(0, "ok"), rel(0, "invoke"), rel(0, "ok"),
                acq(1, "invoke"), acq(1, "ok")]) == A.VALID
    # two acquires that both succeed without a release in between
    assert run([acq(0, "invoke"), acq(0, "ok"), acq(1, "invoke"), acq(1, "ok")]) == A.INVALID
    # a crashed release may have happened
    assert run([acq(0, "invoke"), acq(0, "ok"), rel(0, "invoke"), rel(0, "info"),
                acq(1, "invoke"), acq(1, "ok")]) == A.VALID
    # releasing a free lock
    assert run([rel(0, "invoke"), rel(0, "ok")]) == A.INVALID


def test_register_and_unknown_ops():
    h = [{"process": 0, "type": "invoke", "f": "write", "value": 1},
         {"process": 0, "type": "ok", "f": "write", "value": 1},
         {"process": 1, "type": "invoke", "f": "read", "value": None},
         {"process": 1, "type": "ok", "f": "read", "value": 1}]
    assert M.to_device_ops(M.register(0), h) == h
    with pytest.raises(ValueError):
        M.to_device_ops(M.register(0), h + [{"process": 2, "type": "invoke", "f": "cas",
                                             "value": [1, 2]}])
    with pytest.raises(ValueError):
        M.to_device_ops(M.mutex(), [{"process": 0, "type": "invoke", "f": "read", "value": None}])
    # nemesis ops pass through untouched
    nem = {"process": "nemesis", "type": "info", "f": "start", "value": None}
    assert M.to_device_ops(M.mutex(), [nem]) == [nem]
    # independent tuples keep their key
    t = M.to_device_ops(M.mutex(), [{"process": 0, "type": "invoke", "f": "acquire",
                                     "value": H.tuple_("k", None)}])
    assert H.is_tuple(t[0]["value"]) and t[0]["value"].key == "k" and t[0]["value"].val == [0, 1]
    assert M.Register(3).step({"f": "read", "value": 3}) == M.Register(3)
    assert M.is_inconsistent(M.Mutex(True).step({"f": "acquire"}))


def test_final_paths_end_inconsistent(built):
    """:final-paths (checker.clj:146-158) built from the frontier's
    configurations: each path starts at a configuration's model and ends in
    the failing :op, whose step from that model is inconsistent, with the
    knossos message text (nil prints as nothing: Clojure's str)."""
    import json
    import os
    from jepsen_amd import checker
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "perf_test.json")))
    cols = H.encode(d["history"])
    r = oracle.check_cas_full(cols, init=A.NIL)
    assert r["valid"] == A.INVALID
    out = checker.lin_result(r["valid"], r["cause"], r["fail_entry"], r["explored"], cols,
                             r["previous_ok"], r["last_op"], r["analyzer"])
    checker.add_configs(out, oracle.lin_configs(cols, [0], init=A.NIL)[0], cols, M.CASRegister(None))
    assert 0 < len(out["final-paths"]) == len(out["configs"]) <= 10
    for cfg, p in zip(out["configs"], out["final-paths"]):
        # knossos' Config record [K]: model, last-op, pending
        assert set(cfg) == {"model", "last-op", "pending"}
        assert all(op["type"] == "invoke" for op in cfg["pending"])
        assert [o["index"] for o in cfg["pending"]] == sorted(o["index"] for o in cfg["pending"])
        # from the configuration through consistent pending steps to the failing op
        assert p[0]["op"] == cfg["last-op"] and p[0]["model"] == cfg["model"] and p[-1]["op"] == out["op"]
        m = M.CASRegister(cfg["model"]["value"])
        for st in p[1:-1]:
            assert st["op"] in cfg["pending"]
            m = m.step(st["op"])
            assert not M.is_inconsistent(m) and st["model"] == {"value": m.value}
        assert M.is_inconsistent(m.step(out["op"]))
        assert p[-1]["model"] == {"inconsistent": m.step(out["op"]).msg}
    assert M.CASRegister(1).step({"f": "cas", "value": [2, None]}).msg == "can't CAS 1 from 2 to "


def test_linear_svg_render(built, tmp_path):
    """checker.clj:146-153: an invalid result is rendered to linear.svg under
    the store path and (:subdirectory opts); no store dir, no file; a
    rendering error is logged, not raised."""
    import json
    import os
    from jepsen_amd import checker, report
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "perf_test.json")))
    cols = H.encode(d["history"])
    r = oracle.check_cas_full(cols, init=A.NIL)
    out = checker.lin_result(r["valid"], r["cause"], r["fail_entry"], r["explored"], cols,
                             r["previous_ok"], r["last_op"], r["analyzer"])
    checker.add_configs(out, oracle.lin_configs(cols, [0], init=A.NIL)[0], cols, M.CASRegister(None))
    p = report.maybe_render({"store-dir": str(tmp_path)}, {"subdirectory": ["independent", 7]}, cols, out)
    assert p == os.path.join(str(tmp_path), "independent", "7", "linear.svg")
    svg = open(p).read()
    assert svg.startswith("<svg") and svg.rstrip().endswith("</svg>")
    assert "can&apos;t read 0 from register" in svg or "can't read 0 from register" in svg
    assert report.maybe_render({}, {}, cols, out) is None
    assert report.maybe_render({"store-dir": str(tmp_path)}, {}, cols, {"valid?": False}) is None
