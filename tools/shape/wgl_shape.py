"""Shape of heavy keys' WGL searches on the CPU (tools/shape/wgl_shape.c):
path length, the dead subtrees hanging off the final path, their sizes and
depths. python tools/shape/wgl_shape.py <seed-rank> key [key ...]"""
import ctypes as C
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
rank = int(sys.argv[1]); keys = [int(k) for k in sys.argv[2:]]
wl = WORKLOADS["c3"]
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"] + 7919 * rank, **wl["gen"])
h = A.make_history(cols)
p64 = C.POINTER(C.c_int64)
for key in keys:
    sel = np.nonzero((cols.key == key) | (cols.key < 0))[0].astype(np.int64)
    out = np.zeros(8, np.int64); cap = 1 << 20
    ds, dd, dp, dt = (np.zeros(cap, np.int64) for _ in range(4))
    L.wgl_shape(C.byref(h), sel.ctypes.data_as(p64), C.c_int64(len(sel)), C.c_int64(A.NIL), C.c_int64(wl["budget"]),
                out.ctypes.data_as(p64), ds.ctypes.data_as(p64), dd.ctypes.data_as(p64), dp.ctypes.data_as(p64), dt.ctypes.data_as(p64), C.c_int64(cap))
    nd = int(out[4]); ds, dd, dp, dt = ds[:nd], dd[:nd], dp[:nd], dt[:nd]
    o = np.argsort(-ds)
    print(f"key {key}: verdict {out[0]} inserts {out[1]} path {out[2]} n_ok {out[5]} maxw {out[6]} ops {out[7]} "
          f"dead subtrees {nd} (sum {ds.sum()}), sizes p50 {np.median(ds) if nd else 0:.0f} p90 {np.percentile(ds, 90) if nd else 0:.0f} "
          f"max {ds.max() if nd else 0}, depth max {dd.max() if nd else 0}")
    print("  largest:", [(int(ds[i]), int(dd[i]), int(dp[i]), int(dt[i])) for i in o[:12]], "(size, depth, at path depth, layer span)")
    big = ds >= 256
    print(f"  subtrees >= 256: {big.sum()} holding {ds[big].sum()}; depth-weighted critical path if all ran at once: "
          f"{out[2] + (dd.max() if nd else 0)} steps vs {out[1]} sequential")
