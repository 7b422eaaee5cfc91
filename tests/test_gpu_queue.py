"""(checker/queue (model/unordered-queue)) and (checker/total-queue) on the
device (jh_check_queue / jh_check_total_queue) against the reference's own
known answers (checker_test.clj:13-88, tests/golden/queue.json) and the CPU
oracle (oracle/queue.py) on seeded synthetic histories."""
import json
import os

import pytest

from conftest import GOLD
from jepsen_amd import checker, model, synth
from oracle import queue as Q

pytestmark = pytest.mark.gpu


def ms(pairs):
    return {v: c for v, c in pairs}


def test_queue_known_answers(ctx):
    d = json.load(open(os.path.join(GOLD, "queue.json")))
    for c in d["queue"]:
        m = None if c["model"] is None else model.unordered_queue()
        assert checker.queue(m).check({}, c["history"], {})["valid?"] == c["valid?"], c["name"]


def test_total_queue_known_answers(ctx):
    d = json.load(open(os.path.join(GOLD, "queue.json")))
    for c in d["total_queue"]:
        got = checker.total_queue().check({}, c["history"], {})
        if c["expected"] is None:
            assert got["valid?"] is True and got["attempt-count"] == 0
            continue
        for k, v in c["expected"].items():
            if k in ("lost", "unexpected", "duplicated", "recovered"):
                assert dict(got[k]) == ms(v), (c["name"], k)
            else:
                assert got[k] == v, (c["name"], k)


def _same_total(got, want):
    for k, v in want.items():
        assert (dict(got[k]) if k in ("lost", "unexpected", "duplicated", "recovered") else got[k]) == \
            (dict(v) if hasattr(v, "items") else v), k


@pytest.mark.parametrize("seed,lost,unexp,dup,rep", [(0, 0, 0, 0, 0), (1, 7, 0, 0, 0), (2, 0, 5, 0, 0),
                                                     (3, 0, 0, 6, 3), (4, 3, 2, 4, 10)])
def test_synthetic_vs_oracle(ctx, seed, lost, unexp, dup, rep):
    cols = synth.queue_history(n_enqueues=3000, n_lost=lost, n_unexpected=unexp, n_duplicated=dup,
                               n_repeat=rep, seed=seed)
    ops = synth.queue_columns_to_ops(cols)
    _same_total(checker.total_queue().check({}, ops, {}), Q.total_queue(ops))
    _same_total(checker.total_queue().check({}, cols, {}), Q.total_queue(ops))
    want = Q.queue(ops)
    got = checker.queue(model.unordered_queue()).check({}, ops, {})
    assert got["valid?"] == want["valid?"]
    if want["valid?"]:
        assert dict(got["final-queue"]) == dict(want["final-queue"])
    else:
        assert got["fail-entry"] == want["fail-index"] and got["error"] == want["error"]


def test_queue_model_failure_row(ctx):
    """An unexpected :ok :dequeue in the middle: the first refused row, and
    the model keeps refusing after it (the first failure is reported)."""
    h = [{"process": 0, "type": "invoke", "f": "enqueue", "value": 1},
         {"process": 0, "type": "ok", "f": "enqueue", "value": 1},
         {"process": 1, "type": "invoke", "f": "dequeue", "value": None},
         {"process": 1, "type": "ok", "f": "dequeue", "value": 1},
         {"process": 1, "type": "invoke", "f": "dequeue", "value": None},
         {"process": 1, "type": "ok", "f": "dequeue", "value": 1},
         {"process": 1, "type": "invoke", "f": "dequeue", "value": None},
         {"process": 1, "type": "ok", "f": "dequeue", "value": 9}]
    got = checker.queue(model.unordered_queue()).check({}, h, {})
    assert got == {"valid?": False, "error": "can't dequeue 1", "fail-entry": 5}
    assert Q.queue(h)["fail-index"] == 5


def test_large_vs_oracle(ctx):
    cols = synth.queue_history(n_enqueues=400_000, n_procs=8, n_lost=50, n_unexpected=20,
                               n_duplicated=30, n_repeat=100, drain_parts=5, seed=9)
    ops = synth.queue_columns_to_ops(cols)
    _same_total(checker.total_queue().check({}, cols, {}), Q.total_queue(ops))
    want = Q.queue(ops)
    r = ctx.check_queue(cols)
    if want["valid?"]:
        assert r["valid"] == 0 and ms(r["final_queue"].tolist()) == dict(want["final-queue"])
    else:
        assert r["valid"] == 2 and r["fail_entry"] == want["fail-index"]


def test_edge_cases(ctx):
    tq = checker.total_queue()
    # nil and keyword values, a drain, a :fail drain (skipped)
    h = [{"process": 0, "type": "invoke", "f": "enqueue", "value": "a"},
         {"process": 0, "type": "ok", "f": "enqueue", "value": "a"},
         {"process": 1, "type": "invoke", "f": "dequeue", "value": None},
         {"process": 1, "type": "ok", "f": "dequeue", "value": None},
         {"process": 2, "type": "invoke", "f": "drain", "value": None},
         {"process": 2, "type": "fail", "f": "drain", "value": None},
         {"process": 2, "type": "invoke", "f": "drain", "value": None},
         {"process": 2, "type": "ok", "f": "drain", "value": ["a", "b"]}]
    _same_total(tq.check({}, h, {}), Q.total_queue(h))
    # a crashed drain throws in the reference; check-safe turns it into :unknown
    bad = h[:7] + [dict(h[7], type="info")]
    r = checker.check_safe(tq, {}, bad, {})
    assert r["valid?"] == "unknown" and "crashed drain" in r["error"]
