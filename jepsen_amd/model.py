"""Models for the linearizability checker (knossos.model, used at
jepsen/src/jepsen/checker.clj:17-23 and the call sites of checker/linearizable).

Only the cas-register is on the device path (BASELINE.json north_star); its
`step` here is the reference semantics, restated from the CASRegister text
quoted at doc/tutorial/04-checker.md:58-72, for documentation and for
host-side single-op use. The device kernel implements the same rules on
interned integer states.
"""
from dataclasses import dataclass
from typing import Any


@dataclass(frozen=True)
class Inconsistent:
    msg: str


def inconsistent(msg):
    return Inconsistent(msg)


def is_inconsistent(m):
    return isinstance(m, Inconsistent)


def _s(v):
    """Clojure's str of a value inside a message: nil prints as nothing,
    vectors as [a b]."""
    if v is None:
        return ""
    if isinstance(v, (list, tuple)):
        return "[" + " ".join("nil" if x is None else _s(x) for x in v) + "]"
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


@dataclass(frozen=True)
class CASRegister:
    """knossos.model/->CASRegister (perf_test.clj:134 uses (->CASRegister 0))."""
    value: Any = None

    def step(self, op):
        f, v = op.get("f"), op.get("value")
        if f == "write":
            return CASRegister(v)
        if f == "cas":
            cur, new = v
            if cur == self.value:
                return CASRegister(new)
            return inconsistent(f"can't CAS {_s(self.value)} from {_s(cur)} to {_s(new)}")
        if f == "read":
            if v is None or v == self.value:
                return self
            return inconsistent(f"can't read {_s(v)} from register {_s(self.value)}")
        raise ValueError(f"No matching clause: {f}")


def cas_register(value=None):
    """(knossos.model/cas-register) / (cas-register v)."""
    return CASRegister(value)


@dataclass(frozen=True)
class Register:
    """knossos.model/register (used as (model/register 0) at
    raftis/src/jepsen/raftis.clj:121): a read/write register. knossos 0.3.4 is
    not vendored; its step is the cas-register's read and write (restated
    from doc/tutorial/04-checker.md:58-72) and any other :f has no clause.
    Parity unpinned: no reference test exercises it."""
    value: Any = None

    def step(self, op):
        if op.get("f") == "cas":
            raise ValueError("No matching clause: cas")
        r = CASRegister(self.value).step(op)
        return r if is_inconsistent(r) else Register(r.value)


def register(value=None):
    return Register(value)


@dataclass(frozen=True)
class Mutex:
    """knossos.model/mutex (used at hazelcast/src/jepsen/hazelcast.clj:675,684):
    :acquire when free takes the lock, :release when held frees it, anything
    else is inconsistent. Parity unpinned (knossos is not vendored)."""
    locked: bool = False

    @property
    def value(self):
        # the device searches it as a cas-register over {0 free, 1 held}
        return 1 if self.locked else 0

    def step(self, op):
        f = op.get("f")
        if f == "acquire":
            return inconsistent("already held") if self.locked else Mutex(True)
        if f == "release":
            return Mutex(False) if self.locked else inconsistent("not held")
        raise ValueError(f"No matching clause: {f}")


def mutex():
    return Mutex()


@dataclass(frozen=True)
class UnorderedQueue:
    """knossos.model/unordered-queue (checker_test.clj:18-33, disque.clj:305,
    rabbitmq_test.clj:56): a multiset of pending values; :enqueue adds its
    value, :dequeue removes one copy or the model is inconsistent ("can't
    dequeue v"). knossos 0.3.4 is not vendored: restated; checked on the
    device by jh_check_queue."""
    pending: tuple = ()

    def step(self, op):
        from collections import Counter
        c = Counter(dict(self.pending))
        f, v = op.get("f"), op.get("value")
        if f == "enqueue":
            c[v] += 1
        elif f == "dequeue":
            if c[v] <= 0:
                return inconsistent("can't dequeue %s" % (v,))
            c[v] -= 1
        else:
            raise ValueError(f"No matching clause: {f}")
        return UnorderedQueue(tuple(sorted(((k, n) for k, n in c.items() if n > 0), key=repr)))


def unordered_queue():
    return UnorderedQueue()


_MUTEX_CAS = {"acquire": [0, 1], "release": [1, 0]}


def to_device_ops(model, history):
    """The op maps the device's cas-register search checks for `model`:
    identity for a cas-register; a register refuses :cas; a mutex is the
    cas-register over {0 free, 1 held} with :acquire = cas 0->1 and :release =
    cas 1->0 (the same transitions as Mutex.step). Independent tuples keep
    their key. Raises ValueError for an :f the model has no clause for, which
    check-safe turns into {:valid? :unknown} as the reference does."""
    if isinstance(model, CASRegister):
        return history
    out = []
    for op in history:
        p = op.get("process")
        client = isinstance(p, int) and not isinstance(p, bool) and p >= 0
        f = op.get("f")
        if isinstance(model, Register):
            if client and f not in ("read", "write"):
                raise ValueError(f"No matching clause: {f}")
            out.append(op)
            continue
        if isinstance(model, Mutex):
            if not client:
                out.append(op)
                continue
            if f not in _MUTEX_CAS:
                raise ValueError(f"No matching clause: {f}")
            o = dict(op)
            o["f"] = "cas"
            v = op.get("value")
            cas = list(_MUTEX_CAS[f])
            if isinstance(v, tuple) and hasattr(v, "key"):     # an independent tuple
                from .history import MapEntry
                o["value"] = MapEntry(v.key, cas)
            else:
                o["value"] = cas
            out.append(o)
            continue
        raise ValueError(f"model {model!r} has no device implementation")
    return out
