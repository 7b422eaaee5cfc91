"""Per-key device timing of the heaviest C3 keys (saved from the rank-0 / rank-6
bench histories under tools/data/), one key per call, on the default phase-2
race and on the workgroup engine (JH_WG=1):  python tools/heavy_keys.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from jepsen_amd import _native  # noqa: E402
from jepsen_amd.history import Columns  # noqa: E402


def load(name):
    z = np.load(os.path.join(ROOT, "tools", "data", name + ".npz"))
    n = len(z["process"])
    return Columns(n=n, process=z["process"], type=z["type"], f=z["f"], key=np.zeros(n, np.int64),
                   value=z["value"], value2=z["value2"], n_keys=1, aux=np.zeros(1, np.int64))


ctx = _native.Context(0)
names = sys.argv[1:] or ["r0_key1086", "r0_key4031", "r0_key4529", "r6_key9152", "r0_key8979"]
for mode in ([os.environ["JH_WG"]] if "JH_WG" in os.environ else ["0", "1"]):
    os.environ["JH_WG"] = mode
    for nm in names:
        cols = load(nm)
        ctx.check_cas_independent(cols)
        t = time.perf_counter()
        v, s = ctx.check_cas_independent(cols)
        wall = (time.perf_counter() - t) * 1e3
        print(f"JH_WG={mode} {nm}: valid={int(v['valid'][0])} explored={int(v['explored'][0])} "
              f"device_ms={s.device_ms:.2f} dfs_ms={s.dfs_ms:.2f} seq_ms={s.seq_ms:.2f} bfs_ms={s.bfs_ms:.2f} "
              f"wall_ms={wall:.1f}", flush=True)
