"""C4's shard (bench.py --workload c4 at N = 1) checked with given jh_lin_opts,
every verdict field against the oracle, mismatching keys printed:
    python tools/c4_parity.py [name=flags:helpers ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _abi as A, _native, shard, synth  # noqa: E402
from oracle import oracle  # noqa: E402

wl = WORKLOADS["c4"]
gcols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"], parts=16, **wl["gen"])
owner = shard.assign_keys(shard.key_costs(gcols), 1)
cols, _, _ = shard.shard_history(gcols, owner, 0)
del gcols
budget = wl["budget"]
ov, _ = oracle.check_cas_independent(cols, budget=budget, threads=16)
ctx = _native.Context(0)
for spec in sys.argv[1:] or ["default=0:0"]:
    name, rest = spec.split("=")
    flags, helpers = (int(x) for x in rest.split(":"))
    kw = {"helpers": helpers} if helpers else {}
    for rep in range(2):
        g, s = ctx.check_cas_independent(cols, budget=budget, flags=flags, **kw)
        bad = np.zeros(len(g), bool)
        for f in A.VERDICT_FIELDS:
            bad |= g[f] != ov[f]
        idx = np.nonzero(bad)[0]
        rows = [{"key": int(k), **{f: [int(g[f][k]), int(ov[f][k])] for f in A.VERDICT_FIELDS if g[f][k] != ov[f][k]}}
                for k in idx[:8]]
        print(json.dumps({"variant": name, "rep": rep, "mismatches": int(len(idx)), "takeovers": int(s.takeovers),
                          "spec_merges": int(s.spec_merges), "first": rows}), flush=True)
