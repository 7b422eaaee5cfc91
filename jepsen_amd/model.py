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
            return inconsistent(f"can't CAS {self.value} from {cur} to {new}")
        if f == "read":
            if v is None or v == self.value:
                return self
            return inconsistent(f"can't read {v} from register {self.value}")
        raise ValueError(f"No matching clause: {f}")


def cas_register(value=None):
    """(knossos.model/cas-register) / (cas-register v)."""
    return CASRegister(value)
