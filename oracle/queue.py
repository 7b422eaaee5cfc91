"""TEST INFRASTRUCTURE ONLY: plain-Python restatements of (checker/queue
(model/unordered-queue)) and (checker/total-queue), the checkers of the
device path in tests/. Only tests/ and bench tools may import it.

  queue        jepsen/src/jepsen/checker.clj:160-180, with knossos 0.3.4's
               unordered-queue model (not vendored: a multiset of pending
               values; :enqueue conj's its value, :dequeue removes one copy or
               the model turns inconsistent)
  total-queue  checker.clj:536-628 (expand-queue-drain-ops :536-568) over
               metametadata/multiset 0.1.1 (intersect = min of counts,
               minus = difference floored at zero; not vendored)

Pinned by the reference's known answers, checker_test.clj:13-88
(tests/golden/queue.json). The inconsistency message of the unordered queue
("can't dequeue v") follows knossos and is parity unpinned.
"""
from collections import Counter


def expand_queue_drain_ops(history):
    """checker.clj:536-568."""
    out = []
    for op in history:
        if op.get("f") != "drain":
            out.append(op)
        elif op.get("type") in ("invoke", "fail"):
            continue
        elif op.get("type") == "ok":
            for e in op.get("value") or ():
                out.append(dict(op, type="invoke", f="dequeue", value=None))
                out.append(dict(op, type="ok", f="dequeue", value=e))
        else:
            raise ValueError("Not sure how to handle a crashed drain operation: %r" % (op,))
    return out


def total_queue(history):
    """checker.clj:570-628. Multisets are Counters."""
    h = expand_queue_drain_ops(history)
    attempts = Counter(o["value"] for o in h if o["type"] == "invoke" and o["f"] == "enqueue")
    enqueues = Counter(o["value"] for o in h if o["type"] == "ok" and o["f"] == "enqueue")
    dequeues = Counter(o["value"] for o in h if o["type"] == "ok" and o["f"] == "dequeue")
    ok = dequeues & attempts
    unexpected = Counter({v: c for v, c in dequeues.items() if v not in attempts})
    duplicated = (dequeues - attempts) - unexpected
    lost = enqueues - dequeues
    recovered = ok - enqueues
    n = lambda m: sum(m.values())
    return {"valid?": not lost and not unexpected,
            "attempt-count": n(attempts), "acknowledged-count": n(enqueues), "ok-count": n(ok),
            "unexpected-count": n(unexpected), "duplicated-count": n(duplicated),
            "lost-count": n(lost), "recovered-count": n(recovered),
            "lost": lost, "unexpected": unexpected, "duplicated": duplicated, "recovered": recovered}


def queue(history, model="unordered-queue"):
    """checker.clj:160-180: reduce the model over the :invoke :enqueue and
    :ok :dequeue ops. Returns the result map plus "fail-index" (the position
    of the failing op in `history`, for the device comparison)."""
    if model is None:
        if history:
            raise TypeError("(queue nil) on a non-empty history: model/step on nil")
        return {"valid?": True, "final-queue": None}
    pending = Counter()
    fail = None
    for i, o in enumerate(history):
        if fail is not None:
            continue          # an inconsistent model steps to itself; the reduce still visits every op
        f, t, v = o.get("f"), o.get("type"), o.get("value")
        if f == "enqueue" and t == "invoke":
            pending[v] += 1
        elif f == "dequeue" and t == "ok":
            if pending[v] > 0:
                pending[v] -= 1
            else:
                fail = {"valid?": False, "error": "can't dequeue %s" % (v,), "fail-index": i}
    return fail if fail is not None else {"valid?": True, "final-queue": +pending}
