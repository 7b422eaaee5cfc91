"""One independent cas-register check of a bench.py workload's history on
cuda:0, for profilers (rocprofv3 --pmc / --kernel-trace wrap this). Prints
the last call's jh_summary as one JSON line (the profiled run's own work:
pmc_traffic.py takes its algorithmic bytes from it).

    python tools/run_once.py c3|c4|c5 [reps] [seed-rank]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _abi as A  # noqa: E402
from jepsen_amd import _native, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
wl = WORKLOADS[name]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
seed = wl["seed"] + 7919 * rank
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=seed, **wl["gen"])
ctx = _native.Context(0)
for _ in range(reps):
    v, s = ctx.check_cas_independent(cols, budget=wl.get("budget"), exact_count=False)   # the timed path
d = {f: (list(getattr(s, f)) if f == "waves" else getattr(s, f)) for f, _ in A.JhSummary._fields_}
d.update(workload=name, seed=seed, entries=int(cols.n))
print("SUMMARY " + json.dumps(d), flush=True)
