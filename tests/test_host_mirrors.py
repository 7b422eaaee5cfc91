"""Host-side result builders of the device checkers (no GPU): the set-full
map from a jh_check_set_full result, and the queue multisets from their
(value, multiplicity) pairs, including interned (keyword) values and nil."""
import numpy as np

from jepsen_amd import _abi as A
from jepsen_amd import checker, history as H


def test_set_full_result_map():
    ops = [{"process": 0, "type": "invoke", "f": "add", "value": 0, "index": 0, "time": 0},
           {"process": 0, "type": "ok", "f": "add", "value": 0, "index": 1, "time": 10},
           {"process": 1, "type": "invoke", "f": "read", "value": None, "index": 2, "time": 20}]
    r = {"valid": A.INVALID, "attempt_count": 3, "stable_count": 1, "lost_count": 1,
         "never_read_count": 1, "stale_count": 1, "lost": np.array([5]), "never_read": np.array([7]),
         "stale": np.array([0]), "has_stable_latencies": 1, "has_lost_latencies": 0,
         "stable_latencies": [0, 1, 2, 3, 4], "lost_latencies": [0] * 5,
         "worst_stale": [(0, 4, 1, 2)]}
    m = checker.set_full_result(r, ops)
    assert m["valid?"] is False and m["lost"] == [5] and m["never-read"] == [7] and m["stale"] == [0]
    assert m["stable-latencies"] == {0: 0, 0.5: 1, 0.95: 2, 0.99: 3, 1: 4}
    assert "lost-latencies" not in m
    w = m["worst-stale"][0]
    assert w["known"] is ops[1] and w["last-absent"] is ops[2] and w["stable-latency"] == 4
    assert m["duplicated-count"] == 0 and m["duplicated"] == {}
    r["valid"] = A.UNKNOWN
    assert checker.set_full_result(r, ops)["valid?"] == "unknown"


def test_queue_multisets_unintern_values():
    h = [{"process": 0, "type": "invoke", "f": "enqueue", "value": "a"},
         {"process": 1, "type": "ok", "f": "dequeue", "value": None},
         {"process": 2, "type": "ok", "f": "drain", "value": ["b", "a"]}]
    cols = H.encode(h, keyed=False)
    assert cols.values_interned and list(cols.f) == [A.F_ENQUEUE, A.F_DEQUEUE, A.F_DRAIN]
    # the drain's elements are interned into aux like scalar values
    o, c = int(cols.value[2]), int(cols.value2[2])
    assert [cols.value_table[x] for x in cols.aux[o:o + c]] == ["b", "a"]
    a_id = cols.value_table.index("a")
    ms = checker._multiset(cols, [(a_id, 2), (A.NIL, 1)])
    assert dict(ms) == {"a": 2, None: 1}


def test_unsupported_inputs_raise_before_the_device():
    """The device checkers refuse what they do not cover (the JVM shim then
    falls back to the reference checker)."""
    import pytest
    from jepsen_amd import model
    with pytest.raises(TypeError):
        checker.set_full().check({}, [{"process": 0, "type": "invoke", "f": "add", "value": "x",
                                       "time": 0}], {})
    with pytest.raises(TypeError):
        checker.queue(model.cas_register()).check({}, [{"process": 0, "type": "invoke",
                                                        "f": "enqueue", "value": 1}], {})
    # (queue nil) on an empty history is valid (checker_test.clj:14-15)
    assert checker.queue(None).check({}, [], {})["valid?"] is True


def test_subhistories_one_pass_equals_subhistory():
    """independent.subhistories (one pass) == subhistory per key
    (independent.clj:234-245), un-keyed and nemesis ops included, in order."""
    from jepsen_amd import independent as IND
    from jepsen_amd import synth
    from jepsen_amd import history as H
    cols, _ = synth.cas_register(n_keys=40, ops_per_key=30, nemesis_every=25, seed=9)
    hist = [H.decode_op(cols, i) for i in range(cols.n)]
    hist.insert(7, {"process": 3, "type": "invoke", "f": "read", "value": None})
    subs = IND.subhistories(hist)
    assert list(subs) == IND.history_keys(hist)
    for k in subs:
        assert subs[k] == IND.subhistory(k, hist)
