"""The queue oracles (oracle/queue.py) against the reference's own known
answers, jepsen/test/jepsen/checker_test.clj:13-88 (tests/golden/queue.json).
No GPU."""
import json
import os

from conftest import GOLD
from oracle import queue as Q


def ms(pairs):
    return {(v if not isinstance(v, list) else tuple(v)): c for v, c in pairs}


def test_queue_known_answers():
    d = json.load(open(os.path.join(GOLD, "queue.json")))
    assert len(d["queue"]) == 5
    for c in d["queue"]:
        assert Q.queue(c["history"], c["model"])["valid?"] == c["valid?"], c["name"]


def test_total_queue_known_answers():
    d = json.load(open(os.path.join(GOLD, "queue.json")))
    for c in d["total_queue"]:
        got = Q.total_queue(c["history"])
        if c["expected"] is None:
            assert got["valid?"] is True
            continue
        exp = c["expected"]
        for k, v in exp.items():
            if k in ("lost", "unexpected", "duplicated", "recovered"):
                assert dict(got[k]) == ms(v), (c["name"], k)
            else:
                assert got[k] == v, (c["name"], k)


def test_drain_expansion():
    h = [{"process": 0, "type": "invoke", "f": "enqueue", "value": 1},
         {"process": 0, "type": "ok", "f": "enqueue", "value": 1},
         {"process": 1, "type": "invoke", "f": "drain", "value": None},
         {"process": 1, "type": "ok", "f": "drain", "value": [1, 7]}]
    r = Q.total_queue(h)
    assert r["valid?"] is False and dict(r["unexpected"]) == {7: 1} and r["ok-count"] == 1
    try:
        Q.total_queue(h[:3] + [dict(h[3], type="info")])
        assert False
    except ValueError:
        pass
