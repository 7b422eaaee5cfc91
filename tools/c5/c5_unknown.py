"""C5's :unknown keys on the CPU: per key the widest
window, crashed ops by :f, distinct values, and how many crashed writes /
cas ops the candidate reduction could drop -- a crashed write or cas whose
result value v no op that can still be linearized after it observes (no
read of v, no cas expecting v, among ops completing after the crashed op's
invocation or crashed themselves). Such an op can always be left
unlinearized: in any linearization that holds it, the ops between it and
the next state change cannot depend on v, so removing it keeps the rest
valid -- a sound reduction that changes no verdict.

    python tools/c5/c5_unknown.py [n_keys]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _abi as A, synth  # noqa: E402
from oracle import oracle  # noqa: E402

wl = WORKLOADS["c5"]
nk = int(sys.argv[1]) if len(sys.argv) > 1 else 200
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"], **wl["gen"])
v = oracle.check_cas_independent_range(cols, 0, nk, threads=8)
order = np.argsort(cols.key, kind="stable")
bounds = np.searchsorted(cols.key[order], np.arange(cols.n_keys + 1))
rows_all = []
stats = []
for k in range(nk):
    rows = order[bounds[k]:bounds[k + 1]]
    open_, ops = {}, []
    for r in rows:
        p, ty = int(cols.process[r]), int(cols.type[r])
        if p < 0:
            continue
        if ty == A.TYPE_INVOKE:
            open_[p] = len(ops)
            ops.append({"call": int(r), "ret": None, "f": int(cols.f[r]), "v": int(cols.value[r]),
                        "v2": int(cols.value2[r]), "fail": False})
        elif ty in (A.TYPE_OK, A.TYPE_FAIL):
            o = ops[open_.pop(p)]
            if ty == A.TYPE_FAIL:
                o["fail"] = True
            else:
                o["ret"] = int(r)
                if o["f"] == A.F_READ and o["v"] == A.NIL:
                    o["v"] = int(cols.value[r])
    ops = [o for o in ops if not o["fail"]]
    crashed = [o for o in ops if o["ret"] is None]
    cf = {"read": sum(o["f"] == A.F_READ for o in crashed), "write": sum(o["f"] == A.F_WRITE for o in crashed),
          "cas": sum(o["f"] == A.F_CAS for o in crashed)}
    vals = {o["v"] for o in ops if o["v"] != A.NIL} | {o["v2"] for o in ops if o["f"] == A.F_CAS}
    droppable = 0
    for w in crashed:
        if w["f"] not in (A.F_WRITE, A.F_CAS):
            continue
        val = w["v"] if w["f"] == A.F_WRITE else w["v2"]
        seen = False
        for o in ops:
            if o is w or not (o["ret"] is None or o["ret"] > w["call"]):
                continue
            if (o["f"] == A.F_READ and o["v"] == val) or (o["f"] == A.F_CAS and o["v"] == val):
                seen = True
                break
        droppable += not seen
    # the widest window: ops open at some :ok return (crashed ones stay open)
    rets = sorted(o["ret"] for o in ops if o["ret"] is not None)
    calls = np.array(sorted(o["call"] for o in ops))
    ends = np.array(sorted((o["ret"] if o["ret"] is not None else 1 << 62) for o in ops))
    maxw = max((int(np.searchsorted(calls, r) - np.searchsorted(ends, r)) for r in rets), default=0)
    stats.append({"key": k, "valid": int(v["valid"][k]) if v is not None else None,
                  "explored": int(v["explored"][k]) if v is not None else None, "max_window": maxw,
                  "crashed": cf, "values": len(vals), "droppable_crashed": droppable, "ops": len(ops)})
unk = [s for s in stats if s["valid"] == A.UNKNOWN]
print(json.dumps({"keys": nk, "unknown": len(unk), "budget": A.DEFAULT_BUDGET,
                  "unknown_with_a_droppable_op": sum(s["droppable_crashed"] > 0 for s in unk),
                  "droppable_ops_total": sum(s["droppable_crashed"] for s in unk),
                  "crashed_writes_cas_total": sum(s["crashed"]["write"] + s["crashed"]["cas"] for s in unk),
                  "median_window_unknown": float(np.median([s["max_window"] for s in unk])) if unk else None,
                  "median_window_decided": float(np.median([s["max_window"] for s in stats if s["valid"] != A.UNKNOWN]))
                  if len(unk) < len(stats) else None}))
for s in unk[:8]:
    print(json.dumps(s))
