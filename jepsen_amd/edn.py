"""History ingest: Jepsen's history.edn into op maps / Columns.

Jepsen writes `history.edn` with one `prn`-printed op map per line
(jepsen/src/jepsen/store.clj:346-357 `write-history!`, through
jepsen/src/jepsen/util.clj:191-213 `pwrite-history!`), e.g.

    {:type :invoke, :f :cas, :value [1 [3 4]], :process 2, :time 12, :index 7}
    {:type :info, :f :start, :value "Cut off", :process :nemesis, :time 19}

`read_history` parses that text (the EDN subset prn emits: maps, vectors,
lists, sets, keywords, symbols, strings, characters, integers, ratios,
floats, nil/true/false, `#tag form` literals, `#_` discards and comments)
into the op dicts of jepsen_amd.history; `load_columns` goes straight to the
columnar encoding the device path consumes.

prn prints a jepsen.independent tuple (a MapEntry, independent.clj:21-29) as
a plain vector, so the text alone cannot tell `[k v]` from a two-element
value: pass independent=True to read the value of every client op as a
tuple, as jepsen.independent/checker sees it.
"""
import re
from fractions import Fraction

from . import history as H


class Keyword(str):
    """An EDN keyword; equal to its name as a str (`:read` == "read")."""
    __slots__ = ()

    def __repr__(self):
        return ":" + str.__str__(self)


class Symbol(str):
    __slots__ = ()

    def __repr__(self):
        return str.__str__(self)


class Tagged:
    """A `#tag form` literal with no reader of its own (kept whole)."""
    __slots__ = ("tag", "form")

    def __init__(self, tag, form):
        self.tag, self.form = tag, form

    def __eq__(self, o):
        return isinstance(o, Tagged) and (self.tag, self.form) == (o.tag, o.form)

    def __hash__(self):
        return hash((self.tag, repr(self.form)))

    def __repr__(self):
        return f"#{self.tag} {self.form!r}"


_TOKEN = re.compile(r'''
    (?P<ws>[\s,]+|;[^\n]*)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<open>\#\{|[\[{(])
  | (?P<close>[\]})])
  | (?P<discard>\#_)
  | (?P<tag>\#[A-Za-z][\w.*+!?$%&=<>/-]*)
  | (?P<char>\\(?:newline|space|tab|return|formfeed|backspace|u[0-9a-fA-F]{4}|.))
  | (?P<num>[+-]?\d+(?:/\d+|\.\d*(?:[eE][+-]?\d+)?M?|[eE][+-]?\d+M?|N|M)?(?=[\s,\]})"\#;]|$))
  | (?P<atom>[^\s,\[\]{}()"\#;]+)
''', re.VERBOSE)

_CHARS = {"newline": "\n", "space": " ", "tab": "\t", "return": "\r", "formfeed": "\f",
          "backspace": "\b"}
_ESC = {"n": "\n", "t": "\t", "r": "\r", "b": "\b", "f": "\f", '"': '"', "\\": "\\", "/": "/"}
_CLOSE = {"[": "]", "{": "}", "(": ")", "#{": "}"}


class EdnError(ValueError):
    pass


def _string(tok):
    body = tok[1:-1]
    if "\\" not in body:
        return body
    out, i = [], 0
    while i < len(body):
        c = body[i]
        if c == "\\":
            e = body[i + 1]
            if e == "u":
                out.append(chr(int(body[i + 2:i + 6], 16)))
                i += 6
                continue
            out.append(_ESC.get(e, e))
            i += 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _number(tok):
    t = tok.rstrip("NM")
    if "/" in t:
        a, b = t.split("/")
        return Fraction(int(a), int(b))
    if any(c in t for c in ".eE") or tok.endswith("M"):
        return float(t)
    return int(t)


def _atom(tok):
    if tok == "nil":
        return None
    if tok == "true":
        return True
    if tok == "false":
        return False
    if tok.startswith(":"):
        return Keyword(tok[1:])
    return Symbol(tok)


class _Reader:
    def __init__(self, text):
        self.toks = []
        pos = 0
        for m in _TOKEN.finditer(text):
            if m.start() != pos:
                raise EdnError(f"unreadable EDN at offset {pos}: {text[pos:pos + 20]!r}")
            pos = m.end()
            if m.lastgroup != "ws":
                self.toks.append((m.lastgroup, m.group()))
        if pos != len(text):
            raise EdnError(f"unreadable EDN at offset {pos}: {text[pos:pos + 20]!r}")
        self.i = 0

    def done(self):
        return self.i >= len(self.toks)

    def form(self):
        if self.i >= len(self.toks):
            raise EdnError("unexpected end of EDN input")
        kind, tok = self.toks[self.i]
        self.i += 1
        if kind == "str":
            return _string(tok)
        if kind == "num":
            return _number(tok)
        if kind == "atom":
            return _atom(tok)
        if kind == "char":
            name = tok[1:]
            if name.startswith("u") and len(name) == 5:
                return chr(int(name[1:], 16))
            return _CHARS.get(name, name)
        if kind == "discard":
            self.form()
            return self.form()
        if kind == "tag":
            form = self.form()
            tag = tok[1:]
            if tag == "inst" or tag == "uuid":
                return form                      # the literal's text
            if isinstance(form, dict):           # a record: #jepsen.history.Op{...}
                return form
            return Tagged(tag, form)
        if kind == "open":
            items = self._seq(_CLOSE[tok])
            if tok == "{":
                if len(items) % 2:
                    raise EdnError("map with an odd number of forms")
                return {(str(items[j]) if isinstance(items[j], Keyword) else items[j]): items[j + 1]
                        for j in range(0, len(items), 2)}
            if tok == "#{":
                return frozenset(items)
            return items
        raise EdnError(f"unexpected {tok!r}")

    def _seq(self, close):
        items = []
        while True:
            if self.i >= len(self.toks):
                raise EdnError(f"missing {close!r}")
            kind, tok = self.toks[self.i]
            if kind == "close":
                if tok != close:
                    raise EdnError(f"expected {close!r}, found {tok!r}")
                self.i += 1
                return items
            if kind == "discard":
                self.i += 1
                self.form()
                continue
            items.append(self.form())


def read_all(text):
    """Every top-level EDN form in `text`."""
    r = _Reader(text)
    out = []
    while not r.done():
        out.append(r.form())
    return out


def _op(m, independent):
    if not isinstance(m, dict):
        raise EdnError(f"a history entry is not a map: {m!r}")
    op = {k: (str(v) if isinstance(v, Keyword) and k in ("type", "f", "process") else v)
          for k, v in m.items()}
    v = op.get("value")
    if independent and isinstance(op.get("process"), int) and isinstance(v, list) and len(v) == 2:
        op["value"] = H.MapEntry(v[0], v[1])
    return op


def read_history(text, independent=False):
    """history.edn text -> op dicts (history order). A file holding one
    vector of op maps (a history literal) reads the same."""
    forms = read_all(text)
    if len(forms) == 1 and isinstance(forms[0], list):
        forms = forms[0]
    return [_op(m, independent) for m in forms]


def load_history(path, independent=False):
    with open(path, encoding="utf-8") as fh:
        return read_history(fh.read(), independent)


def load_columns(path, independent=False, **kw):
    """history.edn -> Columns (include/jh.h layout), keyed by independent tuple
    when independent=True."""
    return H.encode(load_history(path, independent), keyed=independent, **kw)


def prn_op(op):
    """An op map as Jepsen's prn prints it (util.clj prn-op), for fixtures."""
    def f(x):
        if x is None:
            return "nil"
        if x is True:
            return "true"
        if x is False:
            return "false"
        if isinstance(x, Keyword):
            return repr(x)
        if isinstance(x, H.MapEntry) or isinstance(x, (list, tuple)):
            return "[" + " ".join(f(y) for y in x) + "]"
        if isinstance(x, (set, frozenset)):
            return "#{" + " ".join(f(y) for y in sorted(x)) + "}"
        if isinstance(x, dict):
            return "{" + ", ".join(f":{k} {f(v)}" for k, v in x.items()) + "}"
        if isinstance(x, str):
            return '"' + x.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n") + '"'
        return str(x)
    parts = []
    for k, v in op.items():
        if k in ("type", "f") and isinstance(v, str):
            parts.append(f":{k} :{v}")
        elif k == "process" and isinstance(v, str):
            parts.append(f":{k} :{v}")
        else:
            parts.append(f":{k} {f(v)}")
    return "{" + ", ".join(parts) + "}"
