"""Jepsen histories: op maps and their columnar int64 encoding.

A history is a sequence of op maps, as jepsen builds them
(jepsen/src/jepsen/core.clj:305-308 invocations, :204-220 completions,
:266-278 nemesis :info pairs). In Python an op is a dict with the reference's
keyword names as strings:

    {"process": 3, "type": "invoke", "f": "cas", "value": [1, 2]}
    {"process": "nemesis", "type": "info", "f": "start"}
    {"process": 0, "type": "ok", "f": "read", "value": tuple_(7, 3)}

`encode` flattens a history into the columnar layout of include/jh.h
 that the device path consumes.
"""
from dataclasses import dataclass, field
from typing import Any, List, Optional

import numpy as np

from . import _abi as A


class MapEntry(tuple):
    """jepsen.independent/tuple: a clojure.lang.MapEntry [k v]
    (jepsen/src/jepsen/independent.clj:21-29)."""
    __slots__ = ()

    def __new__(cls, k, v):
        return tuple.__new__(cls, (k, v))

    @property
    def key(self):
        return self[0]

    @property
    def val(self):
        return self[1]

    def __repr__(self):
        return f"[{self[0]!r} {self[1]!r}]"


def tuple_(k, v):
    return MapEntry(k, v)


def is_tuple(v):
    return isinstance(v, MapEntry)


TYPES = {"invoke": A.TYPE_INVOKE, "ok": A.TYPE_OK, "fail": A.TYPE_FAIL, "info": A.TYPE_INFO}
TYPE_NAMES = {v: k for k, v in TYPES.items()}
KNOWN_F = {"read": A.F_READ, "write": A.F_WRITE, "cas": A.F_CAS, "add": A.F_ADD,
           "enqueue": A.F_ENQUEUE, "dequeue": A.F_DEQUEUE, "drain": A.F_DRAIN}


def invoke_op(process, f, value):
    return {"process": process, "type": "invoke", "f": f, "value": value}


def ok_op(process, f, value):
    return {"process": process, "type": "ok", "f": f, "value": value}


def fail_op(process, f, value):
    return {"process": process, "type": "fail", "f": f, "value": value}


def info_op(process, f, value):
    return {"process": process, "type": "info", "f": f, "value": value}


def index(history):
    """knossos.history/index (called at jepsen/src/jepsen/core.clj:441)."""
    return [dict(op, index=i) for i, op in enumerate(history)]


@dataclass
class Columns:
    """Columnar history (include/jh.h `jh_history`), host numpy arrays."""
    n: int
    process: np.ndarray
    type: np.ndarray
    f: np.ndarray
    key: np.ndarray
    value: np.ndarray
    value2: np.ndarray
    n_keys: int
    aux: Optional[np.ndarray] = None
    keys: List[Any] = field(default_factory=list)      # key id -> original key
    f_names: List[Any] = field(default_factory=list)   # interned f id - 16 -> name
    values_interned: bool = False                       # scalar values were interned
    value_table: List[Any] = field(default_factory=list)
    ints_only: bool = True                              # every non-nil value is an int

    def as_jh(self):
        return A.make_history(self)


def _is_int(x):
    return isinstance(x, (int, np.integer)) and not isinstance(x, bool)


def encode(history, keyed=True, intern_values=None):
    """Encode op maps into Columns.

    keyed: decode independent tuples into the key column (else key = -1 and
    tuple values are kept whole, i.e. interned).
    intern_values: None = intern scalars only if some value is not an int.
    """
    n = len(history)
    proc = np.empty(n, np.int64)
    typ = np.empty(n, np.int64)
    fcol = np.empty(n, np.int64)
    key = np.full(n, -1, np.int64)
    val = np.full(n, A.NIL, np.int64)
    val2 = np.full(n, A.NIL, np.int64)
    aux: List[int] = []
    key_ids = {}
    keys: List[Any] = []
    f_ids = {}
    f_names: List[Any] = []
    other_procs = {"nemesis": -1}
    raw = []
    ints_only = True
    for i, op in enumerate(history):
        p = op.get("process")
        if _is_int(p) and p >= 0:
            proc[i] = int(p)
        else:
            if p not in other_procs:
                other_procs[p] = -1 - len(other_procs)
            proc[i] = other_procs[p]
        t = op.get("type")
        if t not in TYPES:
            raise ValueError(f"unknown :type {t!r} in op {op!r}")
        typ[i] = TYPES[t]
        f = op.get("f")
        if f in KNOWN_F:
            fcol[i] = KNOWN_F[f]
        else:
            if f not in f_ids:
                f_ids[f] = A.F_FIRST_INTERNED + len(f_names)
                f_names.append(f)
            fcol[i] = f_ids[f]
        v = op.get("value")
        if keyed and is_tuple(v):
            k = v.key
            if k not in key_ids:
                key_ids[k] = len(keys)
                keys.append(k)
            key[i] = key_ids[k]
            v = v.val
        raw.append(v)
        if v is None:
            continue
        if fcol[i] == A.F_CAS and isinstance(v, (list, tuple)) and len(v) == 2:
            for x in v:
                if x is not None and not _is_int(x):
                    ints_only = False
        elif isinstance(v, (list, tuple, set, frozenset)):
            if not all(_is_int(x) for x in v):
                ints_only = False
        elif not _is_int(v):
            ints_only = False

    do_intern = (not ints_only) if intern_values is None else intern_values
    table = []
    tids = {}

    def scalar(x):
        if x is None:
            return A.NIL
        if do_intern:
            hk = (type(x).__name__, x) if not isinstance(x, (list, dict, set)) else (type(x).__name__, repr(x))
            if hk not in tids:
                tids[hk] = len(table)
                table.append(x)
            return tids[hk]
        xi = int(x)
        if xi == A.NIL:
            raise OverflowError("value collides with the nil sentinel")
        return xi

    for i, v in enumerate(raw):
        if v is None:
            continue
        fi = fcol[i]
        if fi == A.F_CAS and isinstance(v, (list, tuple)) and len(v) == 2:
            val[i] = scalar(v[0])
            val2[i] = scalar(v[1])
        elif isinstance(v, (list, tuple, set, frozenset)) and fi in (A.F_READ, A.F_DRAIN):
            # a set read / a drain: its elements go to aux (CSR)
            elems = list(v)
            if isinstance(v, (set, frozenset)):
                try:
                    elems = sorted(v)
                except TypeError:
                    pass
            val[i] = len(aux)
            val2[i] = len(elems)
            aux.extend(scalar(x) for x in elems)
        else:
            val[i] = scalar(v)
    return Columns(n=n, process=proc, type=typ, f=fcol, key=key, value=val, value2=val2,
                   n_keys=len(keys), aux=np.asarray(aux, np.int64) if aux else np.zeros(1, np.int64),
                   keys=keys, f_names=f_names, values_interned=do_intern,
                   value_table=table, ints_only=ints_only)


def decode_op(cols: Columns, i: int):
    """Inverse of encode for one row (for reports and :op fields)."""
    op = {}
    p = int(cols.process[i])
    op["process"] = p if p >= 0 else ("nemesis" if p == -1 else p)
    op["type"] = TYPE_NAMES[int(cols.type[i])]
    fi = int(cols.f[i])
    inv_f = {v: k for k, v in KNOWN_F.items()}
    op["f"] = inv_f.get(fi, cols.f_names[fi - A.F_FIRST_INTERNED] if fi >= A.F_FIRST_INTERNED and
                        fi - A.F_FIRST_INTERNED < len(cols.f_names) else fi)

    def unscalar(x):
        x = int(x)
        if x == A.NIL:
            return None
        return cols.value_table[x] if cols.values_interned else x

    if op["f"] == "cas" and (cols.value[i] != A.NIL or cols.value2[i] != A.NIL):
        v = [unscalar(cols.value[i]), unscalar(cols.value2[i])]
    else:
        v = unscalar(cols.value[i])
    k = int(cols.key[i])
    if k >= 0:
        v = MapEntry(cols.keys[k], v)
    op["value"] = v
    op["index"] = i
    return op
