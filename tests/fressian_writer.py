"""A minimal fressian writer (test infrastructure for tests/test_ingest.py).

No JVM exists here, so test.fressian fixtures are written by this restatement
of org.fressian's FressianWriter as clojure.data.fressian and the reference's
store handlers drive it (jepsen/src/jepsen/store.clj:28-79): keywords as KEY
with their namespace and name through the priority cache, maps as MAP + a
list of k v, vectors as lists, independent tuples as the "map-entry" tag,
sets as the "persistent-hash-set" tag (or SET), ints in fressian's packed
forms, strings packed or length-prefixed. It is only as faithful as that
restatement: files from a real JVM are not available here (parity unpinned).
"""
import struct

from jepsen_amd import edn
from jepsen_amd import history as H


class Writer:
    def __init__(self, set_tag=True):
        self.b = bytearray()
        self.pcache = {}
        self.scache = {}
        self.set_tag = set_tag

    def int_(self, i):
        x = i ^ (i >> 63)
        s = 64 - x.bit_length()
        b = self.b
        if s <= 14:
            b.append(0xF8)
            b += struct.pack(">q", i)
        elif s <= 22:
            b.append(0x7E + (i >> 48))
            b += (i & ((1 << 48) - 1)).to_bytes(6, "big")
        elif s <= 30:
            b.append(0x7A + (i >> 40))
            b += (i & ((1 << 40) - 1)).to_bytes(5, "big")
        elif s <= 38:
            b.append(0x76 + (i >> 32))
            b += (i & 0xFFFFFFFF).to_bytes(4, "big")
        elif s <= 44:
            b.append(0x72 + (i >> 24))
            b += (i & 0xFFFFFF).to_bytes(3, "big")
        elif s <= 51:
            b.append(0x68 + (i >> 16))
            b += (i & 0xFFFF).to_bytes(2, "big")
        elif s <= 57 or i < -1:
            b.append(0x50 + (i >> 8))
            b.append(i & 0xFF)
        else:
            b.append(i & 0xFF)

    def string(self, s):
        u = s.encode("utf-8")
        if len(u) < 8:
            self.b.append(0xDA + len(u))
        else:
            self.b.append(0xE3)
            self.int_(len(u))
        self.b += u

    def cached(self, o):
        if o is None:
            self.b.append(0xF7)
            return
        k = (type(o).__name__, o)
        if k in self.pcache:
            i = self.pcache[k]
            if i < 32:
                self.b.append(0x80 + i)
            else:
                self.b.append(0xCC)
                self.int_(i)
            return
        self.b.append(0xCD)
        self.pcache[k] = len(self.pcache)
        self.obj(o)

    def list_(self, xs):
        xs = list(xs)
        if len(xs) < 8:
            self.b.append(0xE4 + len(xs))
        else:
            self.b.append(0xEC)
            self.int_(len(xs))
        for x in xs:
            self.obj(x)

    def tag(self, t, n):
        if t in self.scache:
            i = self.scache[t]
            if i < 16:
                self.b.append(0xA0 + i)
            else:
                self.b.append(0xF0)
                self.int_(i)
            return
        self.scache[t] = len(self.scache)
        self.b.append(0xEF)
        self.string(t)
        self.int_(n)

    def keyword(self, name):
        ns, _, nm = name.rpartition("/") if "/" in name else (None, None, name)
        self.b.append(0xCA)
        self.cached(ns)
        self.cached(nm)

    def obj(self, x):
        b = self.b
        if x is None:
            b.append(0xF7)
        elif x is True:
            b.append(0xF5)
        elif x is False:
            b.append(0xF6)
        elif isinstance(x, edn.Keyword):
            self.keyword(str(x))
        elif isinstance(x, int):
            self.int_(x)
        elif isinstance(x, float):
            b.append(0xFA)
            b += struct.pack(">d", x)
        elif isinstance(x, str):
            self.string(x)
        elif isinstance(x, H.MapEntry):
            self.tag("map-entry", 2)
            self.obj(x[0])
            self.obj(x[1])
        elif isinstance(x, dict):
            b.append(0xC0)
            kv = []
            for k, v in x.items():
                kv += [edn.Keyword(k) if isinstance(k, str) and not isinstance(k, edn.Keyword) else k, v]
            self.list_(kv)
        elif isinstance(x, (set, frozenset)):
            if self.set_tag:
                self.tag("persistent-hash-set", len(x))
                for e in sorted(x):
                    self.obj(e)
            else:
                b.append(0xC1)
                self.list_(sorted(x))
        elif isinstance(x, (list, tuple)):
            self.list_(x)
        else:
            raise TypeError(f"cannot write {x!r}")


def op_map(op):
    """An op dict (history.py form) as the JVM holds it: keyword :type / :f /
    :process(:nemesis) values."""
    out = {}
    for k, v in op.items():
        if k in ("type", "f") and isinstance(v, str) and not isinstance(v, edn.Keyword):
            v = edn.Keyword(v)
        if k == "process" and isinstance(v, str) and not isinstance(v, edn.Keyword):
            v = edn.Keyword(v)
        out[k] = v
    return out


def test_map(ops, set_tag=True, extra=True):
    """bytes of a test.fressian: {:name .. :start-time .. :history [..] :results ..}"""
    w = Writer(set_tag=set_tag)
    m = {"name": "ingest-test", "start-time": "20261017T120000.000Z"}
    if extra:
        m["nodes"] = ["n1", "n2", "n3"]
        m["concurrency"] = 5
    m["history"] = [op_map(o) for o in ops]
    if extra:
        m["results"] = {"valid?": True, "configs": [{"model": "x", "pending": [1, 2]}]}
    w.obj(m)
    return bytes(w.b)


def history_vector(ops, set_tag=True):
    w = Writer(set_tag=set_tag)
    w.obj([op_map(o) for o in ops])
    return bytes(w.b)
