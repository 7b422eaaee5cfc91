"""One independent cas-register check of a bench.py workload's rank-0 history
on cuda:0, for profilers (rocprofv3 --pmc / --kernel-trace wrap this).

    python tools/run_once.py c3|c4|c5 [reps] [seed-rank]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _native, synth  # noqa: E402

wl = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"] + 7919 * rank, **wl["gen"])
ctx = _native.Context(0)
for _ in range(reps):
    v, s = ctx.check_cas_independent(cols)
print(f"keys={s.n_keys} invalid={s.n_invalid} unknown={s.n_unknown} explored={s.explored} "
      f"device_ms={s.device_ms:.2f} dfs_ms={s.dfs_ms:.2f} seq_ms={s.seq_ms:.2f} bfs_ms={s.bfs_ms:.2f} "
      f"deferred={s.n_deferred} deferred_entries={s.deferred_entries} seq_probes={s.seq_probes}", flush=True)
