"""The CPU oracle pinned to the reference's own known answers.

No GPU. These tests are what make the oracle trustworthy as the checker for
the device path (tests/test_gpu_*.py)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLD, load_npz_cols
from jepsen_amd import _abi as A
from jepsen_amd import history as H
from jepsen_amd import synth
from oracle import oracle


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_perf_test_history_is_linearizable(built):
    """jepsen/test/jepsen/perf_test.clj:13-137: (checker/linearizable
    {:model (model/->CASRegister 0)}) says :valid? true."""
    d = _json("perf_test.json")
    cols = H.encode(d["history"], keyed=False)
    valid, cause, fail, explored = oracle.check_cas(cols, init=0)
    assert valid == A.VALID and cause == 0
    # all three CPU formulations agree, including on the WGL cache size
    r = oracle.key_selftest(cols, init=0)
    assert r["canonical"] == r["list"] == A.VALID
    assert r["canonical_explored"] == r["list_explored"] == explored


def test_perf_test_history_invalid_with_nil_register(built):
    """Same history against (cas-register) (initial nil): the first ok read of
    0 cannot be explained, so it must be invalid -- cross-checked by both WGL
    formulations (parity unpinned against knossos itself)."""
    cols = H.encode(_json("perf_test.json")["history"], keyed=False)
    r = oracle.key_selftest(cols, init=A.NIL)
    assert r["canonical"] == r["list"] == A.INVALID
    assert r["canonical_explored"] == r["list_explored"]


@pytest.mark.parametrize("case", _json("counter.json")["cases"], ids=lambda c: c["name"])
def test_counter_known_answers(built, case):
    """jepsen/test/jepsen/checker_test.clj:90-166, exact :reads / :errors."""
    cols = H.encode(case["history"], keyed=False)
    r = oracle.check_counter(cols)
    exp = case["expected"]
    assert r["reads"].tolist() == exp["reads"]
    reads = r["reads"]
    errs = [t for t in reads.tolist() if not (t[0] <= t[1] <= t[2])]
    assert errs == exp["errors"]
    assert (r["valid"] == A.VALID) == exp["valid?"]
    assert r["n_errors"] == len(exp["errors"])


@pytest.mark.parametrize("case", _json("interval_str.json")["cases"], ids=lambda c: c["expected"])
def test_interval_str_known_answers(built, case):
    """jepsen/test/jepsen/util_test.clj:14-31."""
    assert oracle.interval_str(case["input"]) == case["expected"]
    from jepsen_amd.checker import integer_interval_set_str
    assert integer_interval_set_str(case["input"]) == case["expected"]


def test_independent_known_answer():
    """jepsen/test/jepsen/independent_test.clj:78-97 through the host mirror
    of independent/checker (generic path, inner checker on CPU)."""
    from jepsen_amd import checker, independent
    d = _json("independent.json")
    hist = []
    for op in d["history"]:
        v = op["value"]
        if isinstance(v, dict) and "tuple" in v:
            v = independent.tuple_(*v["tuple"])
        hist.append({"value": v})

    class Even(checker.Checker):
        def check(self, test, history, opts):
            return {"valid?": len(history) % 2 == 0}

    r = checker.check(independent.checker(Even()), {"name": "independent-checker-test"}, hist, {})
    exp = d["expected"]
    assert r["valid?"] == exp["valid?"]
    assert {str(k): v for k, v in r["results"].items()} == exp["results"]
    assert r["failures"] == exp["failures"]
    assert 0 not in r["results"]      # key 0 produced no ops: no result


@pytest.mark.parametrize("name", ["cas_small", "cas_tiny", "cas_init0", "cas_crashy"])
def test_synthetic_fixtures_reproduce(built, name):
    """The oracle reproduces its committed vectors; the generator is deterministic."""
    man = {m["name"]: m for m in _json("manifest.json")["synthetic"]}[name]
    cols, z = load_npz_cols(f"synthetic_{name}.npz")
    init = A.NIL if man["init"] is None else man["init"]
    v, s = oracle.check_cas_independent(cols, init=init)
    assert (v["valid"] == z["valid"]).all()
    assert (v["explored"] == z["explored"]).all()
    assert (v["fail_entry"] == z["fail_entry"]).all()
    regen, truth = synth.cas_register(**man["generator"])
    assert (regen.process == cols.process).all() and (regen.value == cols.value).all()
    # every key without an injected fault is linearizable by construction
    assert not ((z["valid"] == A.INVALID) & (z["injected"] == 0)).any()


def test_synthetic_counter_set_reproduce(built):
    cols, z = load_npz_cols("synthetic_counter.npz")
    r = oracle.check_counter(cols)
    assert (r["reads"] == z["reads"]).all() and r["valid"] == int(z["valid"])
    assert r["first_err_entry"] == int(z["first_err_entry"])
    cols, z = load_npz_cols("synthetic_set.npz")
    r = oracle.check_set(cols)
    assert r["valid"] == int(z["valid"]) and r["first_fail_entry"] == int(z["first_fail_entry"])
    assert (r["runs"][1] == z["runs_lost"]).all()


def test_linear_tutorial_analysis(built):
    """doc/tutorial/04-checker.md:126-138: the :linear analysis the reference
    prints, whole map, built by the host mirror (checker.lin_result +
    add_configs) from the oracle's analysis of the fixture history: one final
    configuration, {:model {:value 1}, :last-op the :ok :write 1 at :index
    151 with its :time, :pending []}, :analyzer :linear, :final-paths ().
    No :explored key: WGL's cache size is the side channel (.explored)."""
    from jepsen_amd import checker
    from jepsen_amd import model as M
    d = _json("linear_tutorial.json")
    cols = H.encode(d["history"], keyed=False)
    keyed = H.encode([dict(o, value=H.tuple_(0, o["value"])) for o in d["history"]], keyed=True)
    lin, _ = oracle.check_cas_independent(keyed, init=A.NIL, algorithm="linear")
    assert int(lin["valid"][0]) == A.VALID and int(lin["analyzer"][0]) == A.ANALYZER_LINEAR
    cf = oracle.lin_configs(cols, [0], init=A.NIL)[0]
    assert cf == [(1, [], [], 151)]
    out = checker.lin_result(A.VALID, 0, -1, int(lin["explored"][0]), cols, analyzer=A.ANALYZER_LINEAR,
                             ops=d["history"])
    checker.add_configs(out, cf, cols, M.cas_register(), ops=d["history"])
    assert out == d["expected"]
    assert out.explored == int(lin["explored"][0]) and "explored" not in out
