"""Which feature of phase 1's quick search predicts a deferred key's
remaining work (round 6): every C3 key's canonical WGL DFS (the device's
order) snapshotted at the hand-over point (2 047 inserts): its deepest layer
so far, the inserts since that layer was reached (the stall), its depth; then
Spearman correlations of candidate estimates with the inserts still to do.
    python tools/shape/order_study.py [rank] [at]"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _abi as A, synth  # noqa: E402

so = os.path.join(HERE, "libwgl_shape.so")
subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-std=gnu11", "-o", so, os.path.join(HERE, "wgl_shape.c"), "-lpthread"])
L = C.CDLL(so)
rank = int(sys.argv[1]) if len(sys.argv) > 1 else 0
at = int(sys.argv[2]) if len(sys.argv) > 2 else 2047
wl = WORKLOADS["c3"]
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"] + 7919 * rank, **wl["gen"])
h = A.make_history(cols)
p64 = C.POINTER(C.c_int64)
order = np.argsort(cols.key, kind="stable")
bounds = np.searchsorted(cols.key[order], np.arange(cols.n_keys + 1))
unk = np.nonzero(cols.key < 0)[0]
rows = []
for k in range(cols.n_keys):
    sel = np.sort(np.concatenate([order[bounds[k]:bounds[k + 1]], unk])).astype(np.int64)
    out = np.zeros(6, np.int64)
    L.wgl_at(C.byref(h), sel.ctypes.data_as(p64), C.c_int64(len(sel)), C.c_int64(A.NIL), C.c_int64(wl["budget"]),
             C.c_int64(at), out.ctypes.data_as(p64))
    if out[0] > at:
        rows.append((k, *out.tolist()))
R = np.array(rows, dtype=np.float64)
tot, tmax, rise, depth, n_ok = R[:, 1], R[:, 2], R[:, 3], R[:, 4], R[:, 5]
rem = tot - at
prog = np.maximum(tmax, 1) / n_ok
stall = at - rise


def spearman(a, b):
    ra, rb = np.argsort(np.argsort(a)), np.argsort(np.argsort(b))
    return float(np.corrcoef(ra, rb)[0, 1])


cands = {"inserts/progress (round 5)": at / prog, "stall": stall, "stall/progress": (stall + 1) / prog,
         "1 - progress": 1 - prog, "depth": depth, "stall*(1-progress)": (stall + 1) * (1 - prog)}
res = {name: spearman(v, rem) for name, v in cands.items()}
top = np.argsort(-rem)[:10]
print(json.dumps({"rank": rank, "at": at, "deferred": len(rows), "spearman_vs_remaining": res,
                  "heaviest": [{"key": int(R[i, 0]), "remaining": int(rem[i]), "stall": int(stall[i]),
                                "progress": round(float(prog[i]), 3),
                                "rank_by_stall": int((stall > stall[i]).sum()),
                                "rank_by_r5_estimate": int(((at / prog) > (at / prog[i])).sum())} for i in top]},
                 indent=1))
