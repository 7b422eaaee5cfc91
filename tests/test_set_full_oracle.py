"""The set-full oracle (oracle/set_full.py) against the reference's own known
answers, jepsen/test/jepsen/checker_test.clj:461-626 (tests/golden/set_full.json).
No GPU."""
import json
import os

from conftest import GOLD
from oracle import set_full as SF


def _norm(x):
    if isinstance(x, dict):
        return {str(k) if not isinstance(k, str) else k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if isinstance(x, float) and x.is_integer():
        return int(x)
    return x


def _qkeys(m):
    for k in ("stable-latencies", "lost-latencies"):
        if k in m:
            m[k] = {("0" if q == 0 else "1" if q == 1 else str(q)): v for q, v in m[k].items()}
    return m


def test_set_full_known_answers():
    d = json.load(open(os.path.join(GOLD, "set_full.json")))
    assert len(d["cases"]) == 14
    for c in d["cases"]:
        got = _qkeys(SF.set_full(c["history"]))
        exp = c["expected"]
        assert _norm(got) == _norm(exp), (c["name"], got, exp)


def test_set_full_linearizable_option():
    """(set-full {:linearizable? true}): stale elements make it invalid."""
    d = json.load(open(os.path.join(GOLD, "set_full.json")))
    c = [x for x in d["cases"] if x["name"].startswith("write, flutter")][0]
    assert SF.set_full(c["history"], linearizable=True)["valid?"] is False
    ok = [x for x in d["cases"] if x["name"].startswith("successful read")][0]
    assert SF.set_full(ok["history"], linearizable=True)["valid?"] is True


def test_set_full_numpy_oracle_matches_op_map_oracle():
    """oracle/set_full_np.py (columnar, vectorised) == oracle/set_full.py on
    seeded synthetic histories with lost and stale elements."""
    from jepsen_amd import synth
    from oracle import set_full_np as SN
    for seed, (nl, nst, lin) in enumerate([(0, 0, False), (5, 7, False), (0, 12, True), (20, 0, False)]):
        cols, time = synth.set_full_history(n_adds=600, read_every=4, n_lost=nl, n_stale=nst, seed=seed)
        a = SF.set_full(synth.columns_to_ops(cols, time), linearizable=lin)
        a["worst-stale"] = [(r["element"], r["stable-latency"], r["known"]["index"],
                             r["last-absent"]["index"] if r["last-absent"] else -1) for r in a["worst-stale"]]
        assert a == SN.set_full_cols(cols, time, linearizable=lin), seed
