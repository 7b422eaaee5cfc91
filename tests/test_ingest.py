"""Native history ingest (include/jh_io.h, jepsen_amd/ingest.py): history.edn
and test.fressian -> the columnar layout, held column for column and table
for table to the Python reader + history.encode (no GPU).

Fixtures: the reference's own known-answer histories (tests/golden/, from
perf_test.clj, checker_test.clj, independent_test.clj) printed as
history.edn the way store.clj:346-357 writes it, plus seeded synthetic
histories carrying everything prn emits in an op map (nemesis ops with
strings, keyword and string values, nil, floats, sets, nested :error maps,
comments, a whole-history vector literal, maps spread over several lines).
test.fressian files come from tests/fressian_writer.py (no JVM here: the
fressian side is parity unpinned against a JVM-written file)."""
import json
import os
import random

import numpy as np
import pytest

import fressian_writer as FW
from conftest import GOLD
from jepsen_amd import _abi as A
from jepsen_amd import edn
from jepsen_amd import history as H
from jepsen_amd import ingest
from jepsen_amd._native import JhError


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _text(ops):
    return "\n".join(edn.prn_op(o) for o in ops) + "\n"


def _expected(text, independent):
    return H.encode(edn.read_history(text, independent), keyed=independent)


def _same(a, b, what=""):
    assert a.n == b.n, what
    for c in ("process", "type", "f", "key", "value", "value2"):
        assert np.array_equal(getattr(a, c), getattr(b, c)), f"{what}: column {c}"
    assert a.n_keys == b.n_keys, what
    assert a.values_interned == b.values_interned, what
    na = len(a.aux) if a.aux is not None else 0
    if na > 1 or (b.aux is not None and len(b.aux) > 1):
        assert np.array_equal(a.aux, b.aux), f"{what}: aux"
    assert list(a.keys) == list(b.keys), f"{what}: keys"
    assert [type(k) for k in a.keys] == [type(k) for k in b.keys], f"{what}: key types"
    assert list(a.f_names) == list(b.f_names), f"{what}: f names"
    if a.values_interned:
        assert list(a.value_table) == list(b.value_table), f"{what}: value table"
        assert [type(v) for v in a.value_table] == [type(v) for v in b.value_table], f"{what}: value types"


@pytest.fixture(autouse=True)
def small_chunks(monkeypatch):
    # 4 KiB chunks so that even small texts are split over every thread
    monkeypatch.setattr(ingest, "DEFAULT_MIN_CHUNK", 4096)


def _check_edn(ops_or_text, independent=False, threads=(1, 3, 8)):
    text = ops_or_text if isinstance(ops_or_text, str) else _text(ops_or_text)
    exp = _expected(text, independent)
    for t in threads:
        got = ingest.parse_columns(text, independent=independent, fmt="edn", threads=t)
        _same(got, exp, f"edn threads={t}")
    return exp


def _synthetic(n, seed, independent=False, strings=False, sets=False, floats=False):
    rnd = random.Random(seed)
    ops, open_ = [], {}
    fs = ["read", "write", "cas"] + (["add"] if sets else [])
    for i in range(n):
        if rnd.random() < 0.03:
            ops.append({"type": "info", "f": rnd.choice(["start", "stop"]), "value": rnd.choice(
                [None, "Cut off", ["n1", "n2"], {"n1": ["n2"]}]), "process": "nemesis", "time": i})
            continue
        p = rnd.randrange(12)
        if p in open_:
            f, v = open_.pop(p)
            t = rnd.choice(["ok", "ok", "fail", "info"])
            if f == "read":
                v = rnd.choice([None, rnd.randrange(5)]) if not sets else frozenset(rnd.sample(range(40), rnd.randrange(6)))
            op = {"type": t, "f": f, "value": v, "process": p, "time": i}
            if t == "info" and rnd.random() < 0.5:
                op["error"] = {"type": "timeout", "msg": "a\n\"quoted\" \\ thing", "nodes": ["n1"]}
        else:
            f = rnd.choice(fs)
            v = {"read": None, "write": rnd.randrange(5), "cas": [rnd.randrange(5), rnd.randrange(5)],
                 "add": rnd.randrange(100)}[f]
            if strings and rnd.random() < 0.2:
                v = rnd.choice([edn.Keyword("x"), "y", edn.Keyword("ns/z")]) if f != "cas" else [None, "s"]
            if floats and f == "write" and rnd.random() < 0.3:
                v = rnd.random()
            open_[p] = (f, v)
            op = {"type": "invoke", "f": f, "value": v, "process": p, "time": i}
        if independent and op["type"] != "info" or (independent and op["process"] != "nemesis"):
            k = rnd.choice([rnd.randrange(30), rnd.randrange(30), edn.Keyword("k"), "sk"]) if strings else rnd.randrange(30)
            op["value"] = H.MapEntry(k, op["value"])
        ops.append(op)
    return ops


def test_golden_histories_edn(built):
    """perf_test.clj:13-137 and the six counter answers (checker_test.clj:90-166)
    as history.edn: the native reader gives history.encode's columns."""
    _check_edn(_json("perf_test.json")["history"])
    for case in _json("counter.json")["cases"]:
        _check_edn(case["history"])


def test_set_full_and_queue_goldens_edn(built):
    for case in _json("set_full.json")["cases"]:
        ops = []
        for o in case["history"]:
            o = dict(o)
            if o.get("f") == "read" and isinstance(o.get("value"), list):
                o["value"] = frozenset(o["value"])
            ops.append(o)
        _check_edn(ops)
    q = _json("queue.json")
    for case in q["queue"] + (q["total_queue"] if isinstance(q["total_queue"], list) else []):
        _check_edn(case["history"])


@pytest.mark.parametrize("kw", [dict(), dict(independent=True), dict(strings=True), dict(sets=True),
                                dict(floats=True), dict(independent=True, strings=True)])
def test_synthetic_edn(built, kw):
    ind = kw.get("independent", False)
    ops = _synthetic(3000, seed=len(kw) * 7 + 1, **kw)
    _check_edn(ops, independent=ind)


def test_edn_forms(built):
    """The EDN prn can emit: comments, discards, lists, chars, ratios, bigints,
    #inst/#uuid/record tags, vector-literal files, multi-line maps."""
    text = """; a comment line
{:type :invoke, :f :write, :value 3N, :process 0, :time 1 #_ :discarded}
{:type :ok, :f :write, :value 3, :process 0, :time 2, :when #inst "2026-10-17T00:00:00.000-00:00"}
{:type :invoke, :f :cas, :value (1 2), :process 1}
{:type :fail, :f :cas, :value [1 2], :process 1, :error \\x}
#jepsen.history.Op{:type :invoke, :f :read, :value nil, :process 2}
{:type :ok,
 :f :read,
 :value 3,
 :process 2}
{:type :info, :f :start, :value #uuid "f81d4fae-7dec-11d0-a765-00a0c91e6bf6", :process :nemesis}
"""
    _check_edn(text)
    lit = "[" + "\n ".join(edn.prn_op(o) for o in _synthetic(200, 5)) + "]\n"
    _check_edn(lit)
    # non-integer values interned: ratio, float, keyword, string, nested vector
    text2 = """{:type :invoke, :f :write, :value 1/2, :process 0}
{:type :ok, :f :write, :value 1/2, :process 0}
{:type :invoke, :f :write, :value 2.5, :process 1}
{:type :invoke, :f :write, :value :kw, :process 2}
{:type :invoke, :f :write, :value "kw", :process 3}
{:type :invoke, :f :txn, :value [[:r 1 nil] [:w 2 3]], :process 4}
"""
    _check_edn(text2)
    # fields nobody reads are skipped unbuilt: nesting, chars, tags, discards
    text3 = r"""{:type :invoke, :f :write, :error {:nested [1 2 #{3} (4 "s\"]") \] \space], :t #inst "x"}, :value 3, :process 0}
{:type :ok, :extra #_ 1 2, :f :write, :value 3, :process 0, :index #foo/bar [1 {:a \}}]}
{:type :invoke, :meta #_ #_ 1 2 3, :f :read, :process 1, :value nil}
"""
    _check_edn(text3)


def test_multiline_maps_force_the_sequential_fallback(built):
    """Maps spread over lines: chunk starts land inside forms; the boundary
    check re-parses the rest sequentially and the result is unchanged."""
    ops = _synthetic(4000, 11)
    text = "\n".join(edn.prn_op(o).replace(", ", ",\n  ") for o in ops) + "\n"
    _check_edn(text, threads=(1, 4, 8))


def test_large_threads_agree(built, tmp_path):
    ops = _synthetic(60000, 3, independent=True)
    p = tmp_path / "history.edn"
    p.write_text(_text(ops))
    exp = _expected(p.read_text(), True)
    for t in (1, 2, 8):
        got, tm = ingest.load_columns(p, independent=True, threads=t, with_time=True)
        _same(got, exp, f"file threads={t}")
        assert np.array_equal(tm, np.array([o.get("time", A.NIL) for o in ops], np.int64))


@pytest.mark.parametrize("set_tag", [True, False])
@pytest.mark.parametrize("kw", [dict(), dict(independent=True), dict(strings=True), dict(sets=True)])
def test_fressian_test_map(built, kw, set_tag):
    """test.fressian (store.clj:359-366): the :history of the test map, read
    through fressian's priority and struct caches, gives the same columns as
    the same history read from history.edn."""
    ind = kw.get("independent", False)
    ops = _synthetic(1500, seed=17 + len(kw), **kw)
    if kw.get("sets") and set_tag:
        # the store handler writes the element count as the tag's field count
        # and fressian caches struct types by tag: only one set size per file
        # reads back (a JVM reader is bound the same way)
        for o in ops:
            if isinstance(o.get("value"), frozenset):
                o["value"] = frozenset(range(3))
    exp = _expected(_text(ops), ind)
    data = FW.test_map(ops, set_tag=set_tag)
    _same(ingest.parse_columns(data, independent=ind, fmt="fressian"), exp, "fressian test map")
    _same(ingest.parse_columns(data, independent=ind), exp, "fressian auto-detected")
    vec = FW.history_vector(ops, set_tag=set_tag)
    _same(ingest.parse_columns(vec, independent=ind, fmt="fressian"), exp, "fressian history vector")


def test_fressian_ints_and_strings(built):
    """Every packed int width and long strings round-trip."""
    vals = [0, 1, 63, 64, -1, -2, -64, -65, 255, 4095, -4096, 4096, 2 ** 19 - 1, -(2 ** 19), 2 ** 24,
            2 ** 33 - 1, -(2 ** 33), 2 ** 40, 2 ** 47, -(2 ** 48), 2 ** 62, -(2 ** 63) + 1, 2 ** 63 - 1]
    ops = []
    for i, v in enumerate(vals):
        ops.append({"type": "invoke", "f": "write", "value": v, "process": i})
        ops.append({"type": "ok", "f": "write", "value": v, "process": i})
    got = ingest.parse_columns(FW.test_map(ops), fmt="fressian")
    assert got.value.tolist() == [v for v in vals for _ in (0, 1)]
    ops2 = [{"type": "info", "f": "start", "value": "x" * n, "process": "nemesis"} for n in (0, 7, 8, 300, 70000)]
    ops2 += [{"type": "invoke", "f": "write", "value": 1, "process": 0}]
    got = ingest.parse_columns(FW.test_map(ops2), fmt="fressian")
    assert got.values_interned and got.value_table[:5] == ["x" * n for n in (0, 7, 8, 300, 70000)]


def test_errors(built):
    with pytest.raises(JhError, match="unknown :type"):
        ingest.parse_columns('{:type :bogus, :f :read, :process 0}\n', fmt="edn")
    with pytest.raises(JhError, match="unterminated"):
        ingest.parse_columns('{:type :ok, :f :read, :value "abc, :process 0}\n', fmt="edn")
    with pytest.raises(JhError, match="collection"):
        ingest.parse_columns('{:type :invoke, :f :write, :value [1 2], :process 0}\n', fmt="edn")
    with pytest.raises(JhError, match="no :history"):
        w = FW.Writer()
        w.obj({"name": "x"})
        ingest.parse_columns(bytes(w.b), fmt="fressian")
    with pytest.raises(JhError, match="cannot open"):
        ingest.load_columns("/nonexistent/history.edn")
    got = ingest.parse_columns("", fmt="edn")
    assert got.n == 0


def test_ratio_out_of_range(built):
    """a ratio whose numerator or denominator is outside the int64
    range is an error, as an out-of-range integer is (no silent saturation);
    in range it is interned reduced, as Clojure reads it."""
    big = "9" * 25
    with pytest.raises(JhError, match="int64 range"):
        ingest.parse_columns('{:type :invoke, :f :write, :value %s/3, :process 0}\n' % big, fmt="edn")
    with pytest.raises(JhError, match="int64 range"):
        ingest.parse_columns('{:type :invoke, :f :write, :value 3/%s, :process 0}\n' % big, fmt="edn")
    with pytest.raises(JhError, match="int64 range"):
        ingest.parse_columns('{:type :invoke, :f :write, :value -9223372036854775808/2, :process 0}\n', fmt="edn")
    a = ingest.parse_columns('{:type :invoke, :f :write, :value 4/6, :process 0}\n'
                             '{:type :invoke, :f :write, :value 2/3, :process 1}\n', fmt="edn")
    assert a.value[0] == a.value[1]
