"""Check a few keys of a bench.py workload's history alone (tuning builds:
JH_DEBUG=2 prints each engine's per-key statistics), timing each engine by
itself: the BFS alone (JH_LIN_BFS_ONLY), the default race, no helpers.

    python tools/key_probe.py c3 <seed-rank> key [key ...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _abi as A  # noqa: E402
from jepsen_amd import _native, shard, synth  # noqa: E402

name, rank = sys.argv[1], int(sys.argv[2])
keys = [int(k) for k in sys.argv[3:]]
wl = WORKLOADS[name]
seed = wl["seed"] + 7919 * rank
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=seed, **wl["gen"])
own = np.ones(cols.n_keys, np.int64)
own[keys] = 0
sub, mine, _ = shard.shard_history(cols, own, 0)
ctx = _native.Context(0)
budget = int(os.environ.get("JH_PROBE_BUDGET", "0")) or wl.get("budget")
# the checkers' path (no count pass for BFS-settled valid keys) unless "exact"
for label, kw in [("race", {}), ("bfs-only", {"flags": A.LIN_BFS_ONLY}), ("no-helpers", {"flags": A.LIN_NO_HELPERS}),
                  ("exact", {"exact_count": True}), ("race", {})]:
    kw.setdefault("exact_count", False)
    # JH_PROBE_FLAGS: extra jh_lin_opts flags for every run (e.g. 2048, JH_LIN_NO_SPEC)
    if os.environ.get("JH_PROBE_FLAGS"):
        kw["flags"] = kw.get("flags", 0) | int(os.environ["JH_PROBE_FLAGS"])
    t0 = time.perf_counter()
    v, s = ctx.check_cas_independent(sub, budget=budget, **kw)
    ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"run": label, "keys": mine.tolist(), "wall_ms": round(ms, 3), "device_ms": s.device_ms,
                      "valid": v["valid"].tolist(), "explored": v["explored"].tolist(),
                      "seq_ms": s.seq_ms, "bfs_ms": s.bfs_ms, "n_deferred": s.n_deferred,
                      "spec": [s.spec_jobs, s.spec_dead, s.spec_merges, s.spec_nodes]}), flush=True)
