"""Regenerates tests/golden/ (fixtures = data: inputs and expected outputs).

1. Reference known answers, transcribed from the reference's own tests
   (read as text when /root/reference is present; the committed JSON is what
   the tests use, so the GPU box never needs the reference):
     perf_test.json     jepsen/test/jepsen/perf_test.clj:13-137 (history) and
                        :133-137 (expected :valid? true, model (->CASRegister 0))
     counter.json       jepsen/test/jepsen/checker_test.clj:90-166
     interval_str.json  jepsen/test/jepsen/util_test.clj:14-31
     independent.json   jepsen/test/jepsen/independent_test.clj:78-97
     linear_tutorial.json  doc/tutorial/04-checker.md:126-138 (the printed
                        :linear analysis; its history is elided there and
                        reconstructed here)
2. Seeded synthetic vectors (synthetic_*.npz + manifest.json): small
   histories from jepsen_amd.synth with the CPU oracle's verdicts, each
   cross-checked against the knossos-style WGL and (for tiny keys) brute
   force before being written.

Usage: python tools/make_golden.py
"""
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference/jepsen/test/jepsen"


def parse_edn_ops(text):
    """Parse the flat op maps of perf_test.clj: {:k v, ...} with ints,
    keywords and [a b] vectors."""
    ops = []
    for m in re.finditer(r"\{([^{}]*)\}", text):
        body = m.group(1)
        op = {}
        for km in re.finditer(r":([\w?-]+)\s+(\[[^\]]*\]|:[\w-]+|-?\d+|nil)", body):
            k, v = km.group(1), km.group(2)
            if v.startswith("["):
                v = [int(x) for x in v.strip("[]").split()]
            elif v.startswith(":"):
                v = v[1:]
            elif v == "nil":
                v = None
            else:
                v = int(v)
            op[k] = v
        ops.append(op)
    return ops


def perf_test():
    path = os.path.join(REF, "perf_test.clj")
    src = open(path).read()
    start = src.index("(let [history [") + len("(let [history [")
    end = src.index("]]", start)
    ops = parse_edn_ops(src[start:end])
    assert len(ops) == 120, len(ops)
    return {"source": "jepsen/test/jepsen/perf_test.clj:13-137",
            "model": {"cas-register": 0},
            "expected": {"valid?": True},
            "history": ops}


def counter():
    def inv(p, f, v): return {"process": p, "type": "invoke", "f": f, "value": v}
    def ok(p, f, v): return {"process": p, "type": "ok", "f": f, "value": v}
    def fail(p, f, v): return {"process": p, "type": "fail", "f": f, "value": v}
    cases = [
        ("empty", [], {"valid?": True, "reads": [], "errors": []}),
        ("initial read", [inv(0, "read", None), ok(0, "read", 0)],
         {"valid?": True, "reads": [[0, 0, 0]], "errors": []}),
        ("ignore failed ops", [inv(0, "add", 1), fail(0, "add", 1), inv(0, "read", None), ok(0, "read", 0)],
         {"valid?": True, "reads": [[0, 0, 0]], "errors": []}),
        ("initial invalid read", [inv(0, "read", None), ok(0, "read", 1)],
         {"valid?": False, "reads": [[0, 1, 0]], "errors": [[0, 1, 0]]}),
        ("interleaved concurrent reads and writes",
         [inv(0, "read", None), inv(1, "add", 1), inv(2, "read", None), inv(3, "add", 2),
          inv(4, "read", None), inv(5, "add", 4), inv(6, "read", None), inv(7, "add", 8),
          inv(8, "read", None), ok(0, "read", 6), ok(1, "add", 1), ok(2, "read", 0),
          ok(3, "add", 2), ok(4, "read", 3), ok(5, "add", 4), ok(6, "read", 100),
          ok(7, "add", 8), ok(8, "read", 15)],
         {"valid?": False, "reads": [[0, 6, 15], [0, 0, 15], [0, 3, 15], [0, 100, 15], [0, 15, 15]],
          "errors": [[0, 100, 15]]}),
        ("rolling reads and writes",
         [inv(0, "read", None), inv(1, "add", 1), ok(0, "read", 0), inv(0, "read", None),
          ok(1, "add", 1), inv(1, "add", 2), ok(0, "read", 3), inv(0, "read", None),
          ok(1, "add", 2), ok(0, "read", 5)],
         {"valid?": False, "reads": [[0, 0, 1], [0, 3, 3], [1, 5, 3]], "errors": [[1, 5, 3]]}),
    ]
    if os.path.exists(os.path.join(REF, "checker_test.clj")):
        src = open(os.path.join(REF, "checker_test.clj")).read()
        for name, _, _ in cases:
            assert f'(testing "{name}"' in src, name
    return {"source": "jepsen/test/jepsen/checker_test.clj:90-166",
            "cases": [{"name": n, "history": h, "expected": e} for n, h, e in cases]}


def interval_str():
    cases = [([], "#{}"), ([1], "#{1}"), ([1, 2], "#{1..2}"), ([1, 2, 3], "#{1..3}"),
             ([1, 3, 5], "#{1 3 5}"), ([1, 2, 3, 5, 7, 8, 9], "#{1..3 5 7..9}")]
    if os.path.exists(os.path.join(REF, "util_test.clj")):
        src = open(os.path.join(REF, "util_test.clj")).read()
        for _, s in cases:
            assert f'"{s}"' in src, s
    return {"source": "jepsen/test/jepsen/util_test.clj:14-31",
            "cases": [{"input": i, "expected": s} for i, s in cases]}


def independent():
    # (sequential-generator [0 1 2 3] (fn [k] (map (partial array-map :value) (range k))))
    # run by threads [:a :b :c], plus one un-sharded op; an even-checker inner
    ops = [{"value": "not-sharded"}]
    for k in [0, 1, 2, 3]:
        for v in range(k):
            ops.append({"value": {"tuple": [k, v]}})
    return {"source": "jepsen/test/jepsen/independent_test.clj:78-97",
            "inner": "even-checker: {:valid? (even? (count history))}",
            "history": ops,
            "expected": {"valid?": False,
                         "results": {"1": {"valid?": True}, "2": {"valid?": False},
                                     "3": {"valid?": True}},
                         "failures": [2]}}


def synthetic():
    from jepsen_amd import synth
    from jepsen_amd import _abi as A
    from oracle import oracle
    manifest = []
    specs = [
        # name, generator kwargs, init
        ("cas_small", dict(n_keys=300, ops_per_key=40, threads_per_key=6, readers=2, groups=6,
                           p_info=0.05, p_invalid=0.15, nemesis_every=50, seed=101), None),
        ("cas_tiny", dict(n_keys=400, ops_per_key=6, threads_per_key=3, readers=1, groups=5,
                          p_info=0.15, p_invalid=0.3, nemesis_every=7, seed=102), None),
        ("cas_init0", dict(n_keys=200, ops_per_key=60, threads_per_key=10, readers=5, groups=4,
                           p_info=0.02, p_invalid=0.1, nemesis_every=100, seed=103, init_nil=False), 0),
        ("cas_crashy", dict(n_keys=100, ops_per_key=80, threads_per_key=8, readers=3, groups=4,
                            p_info=0.12, p_invalid=0.1, nemesis_every=40, seed=104), None),
    ]
    for name, kw, init in specs:
        cols, truth = synth.cas_register(**kw)
        ini = A.NIL if init is None else init
        v, s = oracle.check_cas_independent(cols, init=ini, mode=0)
        v2, _ = oracle.check_cas_independent(cols, init=ini, mode=3)   # faithful split + list WGL
        assert (v["valid"] == v2["valid"]).all() and (v["explored"] == v2["explored"]).all(), name
        np.savez_compressed(os.path.join(GOLD, f"synthetic_{name}.npz"),
                            process=cols.process, type=cols.type, f=cols.f, key=cols.key,
                            value=cols.value, value2=cols.value2, n_keys=cols.n_keys,
                            valid=v["valid"], cause=v["cause"], fail_entry=v["fail_entry"],
                            explored=v["explored"], injected=truth)
        manifest.append({"name": name, "generator": kw, "init": init, "n": int(cols.n),
                         "n_keys": int(cols.n_keys), "n_invalid": int(s.n_invalid),
                         "n_unknown": int(s.n_unknown), "explored": int(s.explored)})
    # counter and set vectors
    c = synth.counter(n_ops=20000, n_procs=10, read_every=20, p_fail=0.05, p_info=0.02,
                      n_bad_reads=5, seed=105)
    rc = oracle.check_counter(c)
    np.savez_compressed(os.path.join(GOLD, "synthetic_counter.npz"), process=c.process, type=c.type,
                        f=c.f, value=c.value, value2=c.value2, reads=rc["reads"],
                        valid=rc["valid"], n_errors=rc["n_errors"],
                        first_err_entry=rc["first_err_entry"])
    manifest.append({"name": "counter", "n": int(c.n), "valid": int(rc["valid"]),
                     "n_reads": int(rc["n_reads"]), "n_errors": int(rc["n_errors"])})
    st = synth.set_history(n_adds=20000, n_procs=10, p_fail=0.05, p_info=0.02, n_lost=20,
                           n_unexpected=5, seed=106)
    rs = oracle.check_set(st)
    np.savez_compressed(os.path.join(GOLD, "synthetic_set.npz"), process=st.process, type=st.type,
                        f=st.f, value=st.value, value2=st.value2, aux=st.aux,
                        counts=np.array([rs["attempt_count"], rs["acknowledged_count"], rs["ok_count"],
                                         rs["lost_count"], rs["recovered_count"],
                                         rs["unexpected_count"]]),
                        valid=rs["valid"], first_fail_entry=rs["first_fail_entry"],
                        runs_ok=rs["runs"][0], runs_lost=rs["runs"][1],
                        runs_unexpected=rs["runs"][2], runs_recovered=rs["runs"][3])
    manifest.append({"name": "set", "n": int(st.n), "valid": int(rs["valid"]),
                     "lost": int(rs["lost_count"]), "unexpected": int(rs["unexpected_count"])})
    return manifest


def set_full():
    """jepsen/test/jepsen/checker_test.clj:461-626 (set-full-test), transcribed:
    the op bindings of each `let`, the histories given to `c`, and the
    expected maps. `history` (checker_test.clj:448-459) indexes the ops and
    gives op i the time i * 10^6 ns."""
    def op(p, t, f, v):
        return {"process": p, "type": t, "f": f, "value": v}

    def hist(ops):
        return [dict(o, index=i, time=i * 1000000) for i, o in enumerate(ops)]

    lat = lambda x: {"0": x, "0.5": x, "0.95": x, "0.99": x, "1": x}
    base = {"lost": [], "lost-count": 0, "never-read": [], "never-read-count": 0,
            "stale-count": 0, "stale": [], "worst-stale": [], "stable-count": 0,
            "duplicated-count": 0, "duplicated": {}}
    cases = []

    def case(name, line, ops_list, expected):
        for i, ops in enumerate(ops_list):
            cases.append({"name": f"{name}#{i}", "source": f"checker_test.clj:{line}",
                          "history": hist(ops), "expected": dict(base, **expected)})

    a, a_ = op(0, "invoke", "add", 0), op(0, "ok", "add", 0)
    case("never read", 465, [[a, a_]],
         {"attempt-count": 1, "never-read": [0], "never-read-count": 1, "valid?": "unknown"})
    r, rp, rm = op(1, "invoke", "read", None), op(1, "ok", "read", [0]), op(1, "ok", "read", [])
    case("never confirmed, never read", 485, [[a, r, rm]],
         {"attempt-count": 1, "never-read": [0], "never-read-count": 1, "valid?": "unknown"})
    case("successful read either concurrently or after", 499,
         [[r, a, rp, a_], [r, a, a_, rp], [a, r, rp, a_], [a, r, a_, rp], [a, a_, r, rp]],
         {"valid?": True, "attempt-count": 1, "stable-count": 1, "stable-latencies": lat(0)})
    case("Absent read after", 520, [[a, a_, r, rm]],
         {"valid?": False, "attempt-count": 1, "lost": [0], "lost-count": 1,
          "lost-latencies": lat(0)})
    case("Absent read concurrently", 536,
         [[r, a, rm, a_], [r, a, a_, rm], [a, r, rm, a_], [a, r, a_, rm]],
         {"valid?": "unknown", "attempt-count": 1, "never-read": [0], "never-read-count": 1})
    a0, a0_ = op(0, "invoke", "add", 0), op(0, "ok", "add", 0)
    a1, a1_ = op(1, "invoke", "add", 1), op(1, "ok", "add", 1)
    r2, r3 = op(2, "invoke", "read", None), op(3, "invoke", "read", None)
    r2e = op(2, "ok", "read", [])
    r2_0, r3_1 = op(2, "ok", "read", [0]), op(3, "ok", "read", [1])
    r2_1, r2_01 = op(2, "ok", "read", [1]), op(2, "ok", "read", [0, 1])
    case("write, present, missing", 570,
         [[a0, a1, r2, r2_1, a0_, a1_, r2, r2_01, r2, r2_0, r2, r2e]],
         {"valid?": False, "attempt-count": 2, "lost": [0, 1], "lost-count": 2,
          "lost-latencies": {"0": 3, "0.5": 4, "0.95": 4, "0.99": 4, "1": 4}})
    h = [a0, a0_, a1, r2, r2_1, a1_, r2, r3, r3_1, r2_0]
    case("write, flutter, stable/lost", 587, [h],
         {"valid?": False, "attempt-count": 2, "lost": [0], "lost-count": 1,
          "stale-count": 1, "stale": [1],
          "worst-stale": [{"element": 1,
                           "known": dict(r2_1, index=4, time=4000000),
                           "last-absent": dict(r2, index=6, time=6000000),
                           "lost-latency": None, "outcome": "stable", "stable-latency": 2}],
          "stable-count": 1, "lost-latencies": lat(5), "stable-latencies": lat(2)})
    return {"source": "jepsen/test/jepsen/checker_test.clj:448-626", "cases": cases}


def queue():
    """jepsen/test/jepsen/checker_test.clj:13-88 (queue-test, total-queue-test),
    transcribed. knossos.core's invoke-op / ok-op build {:process :type :f
    :value}; keywords become strings; a multiset is a sorted [[value, count]]
    list."""
    def inv(p, f, v): return {"process": p, "type": "invoke", "f": f, "value": v}
    def ok(p, f, v): return {"process": p, "type": "ok", "f": f, "value": v}
    q = [{"name": "empty", "source": "checker_test.clj:14-15", "model": None, "history": [],
          "valid?": True},
         {"name": "Possible enqueue but no dequeue", "source": "checker_test.clj:17-19",
          "model": "unordered-queue", "history": [inv(1, "enqueue", 1)], "valid?": True},
         {"name": "Definite enqueue but no dequeue", "source": "checker_test.clj:21-23",
          "model": "unordered-queue", "history": [ok(1, "enqueue", 1)], "valid?": True},
         {"name": "concurrent enqueue/dequeue", "source": "checker_test.clj:25-29",
          "model": "unordered-queue",
          "history": [inv(2, "dequeue", None), inv(1, "enqueue", 1), ok(2, "dequeue", 1)], "valid?": True},
         {"name": "dequeue but no enqueue", "source": "checker_test.clj:31-33",
          "model": "unordered-queue", "history": [ok(1, "dequeue", 1)], "valid?": False}]
    zero = {"duplicated": [], "lost": [], "unexpected": [], "recovered": []}
    t = [{"name": "empty", "source": "checker_test.clj:36-37", "history": [], "expected": None},
         {"name": "sane", "source": "checker_test.clj:39-58",
          "history": [inv(1, "enqueue", 1), inv(2, "enqueue", 2), ok(2, "enqueue", 2),
                      inv(3, "dequeue", 1), ok(3, "dequeue", 1), inv(3, "dequeue", 2), ok(3, "dequeue", 2)],
          "expected": dict(zero, **{"valid?": True, "recovered": [[1, 1]], "attempt-count": 2,
                                    "acknowledged-count": 1, "ok-count": 2, "unexpected-count": 0,
                                    "lost-count": 0, "duplicated-count": 0, "recovered-count": 1})},
         {"name": "pathological", "source": "checker_test.clj:60-87",
          "history": [inv(1, "enqueue", "hung"), inv(2, "enqueue", "enqueued"), ok(2, "enqueue", "enqueued"),
                      inv(3, "enqueue", "dup"), ok(3, "enqueue", "dup"), inv(4, "dequeue", None),
                      inv(5, "dequeue", None), ok(5, "dequeue", "wtf"), inv(6, "dequeue", None),
                      ok(6, "dequeue", "dup"), inv(7, "dequeue", None), ok(7, "dequeue", "dup")],
          "expected": {"valid?": False, "lost": [["enqueued", 1]], "unexpected": [["wtf", 1]],
                       "recovered": [], "duplicated": [["dup", 1]], "acknowledged-count": 2,
                       "attempt-count": 3, "ok-count": 1, "lost-count": 1, "unexpected-count": 1,
                       "duplicated-count": 1, "recovered-count": 0}}]
    return {"source": "jepsen/test/jepsen/checker_test.clj:13-88", "queue": q, "total_queue": t}


def linear_tutorial():
    """doc/tutorial/04-checker.md:126-138: the analysis (checker/linearizable
    {:model (model/cas-register) :algorithm :linear}) prints for the
    tutorial's etcd register test (:110-124). The tutorial elides the history
    ("..." between its first and last log lines), so the history here is
    reconstructed, seeded: five processes running read / write / cas
    (values 0-4, `gen/cas` of generator.clj:395-403) against a true register
    linearized at invocation, at most two ops in flight, then -- as its last
    log line shows -- process 3's :write 1 alone, ok at :index 151, :time
    14796541900. The expected map is the tutorial's, verbatim (keywords as
    strings, the :configs list as a JSON list)."""
    import random
    rnd = random.Random(20190418)
    hist, reg, t = [], None, 10_000_000
    open_ops = {}
    def emit(op):
        nonlocal t
        t += rnd.randint(1_000_000, 90_000_000)
        op = dict(op, time=t, index=len(hist))
        hist.append(op)
    n_inv = 0
    while n_inv < 75 or open_ops:                   # 75 ops = 150 entries, then drain
        if open_ops and (len(open_ops) >= 2 or n_inv >= 75 or rnd.random() < 0.5):
            p = rnd.choice(sorted(open_ops))
            f, v, res = open_ops.pop(p)
            emit({"process": p, "type": res, "f": f, "value": v})
            continue
        p = rnd.choice([q for q in range(5) if q not in open_ops])
        f = rnd.choice(["read", "write", "cas"])
        n_inv += 1
        if f == "read":
            emit({"process": p, "type": "invoke", "f": f, "value": None})
            open_ops[p] = (f, reg, "ok")
        elif f == "write":
            v = rnd.randint(0, 4)
            emit({"process": p, "type": "invoke", "f": f, "value": v})
            reg = v
            open_ops[p] = (f, v, "ok")
        else:
            v = [rnd.randint(0, 4), rnd.randint(0, 4)]
            emit({"process": p, "type": "invoke", "f": f, "value": v})
            res = "ok" if reg == v[0] else "fail"
            if res == "ok":
                reg = v[1]
            open_ops[p] = (f, v, res)
    assert len(hist) == 150 and not open_ops
    emit({"process": 3, "type": "invoke", "f": "write", "value": 1})
    hist.append({"process": 3, "type": "ok", "f": "write", "value": 1, "index": 151, "time": 14796541900})
    assert hist[-2]["time"] < 14796541900
    expected = {"valid?": True,
                "configs": [{"model": {"value": 1},
                             "last-op": {"process": 3, "type": "ok", "f": "write", "value": 1, "index": 151,
                                         "time": 14796541900},
                             "pending": []}],
                "analyzer": "linear",
                "final-paths": []}
    return {"source": "doc/tutorial/04-checker.md:110-138 (expected map verbatim; history reconstructed)",
            "model": {"cas-register": None}, "algorithm": "linear", "history": hist, "expected": expected}


def main():
    os.makedirs(GOLD, exist_ok=True)
    for name, fn in [("perf_test", perf_test), ("counter", counter), ("interval_str", interval_str),
                     ("independent", independent), ("set_full", set_full),
                     ("queue", queue), ("linear_tutorial", linear_tutorial)]:
        with open(os.path.join(GOLD, name + ".json"), "w") as f:
            json.dump(fn(), f, indent=1)
    man = synthetic()
    with open(os.path.join(GOLD, "manifest.json"), "w") as f:
        json.dump({"generated_by": "tools/make_golden.py", "synthetic": man}, f, indent=1)
    print("wrote", GOLD)


if __name__ == "__main__":
    if "--linear-tutorial" in sys.argv:       # this fixture alone (no reference tree needed)
        with open(os.path.join(GOLD, "linear_tutorial.json"), "w") as f:
            json.dump(linear_tutorial(), f, indent=1)
    else:
        main()
