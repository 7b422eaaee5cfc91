"""One independent cas-register check of the C3 history on cuda:0 (for
profilers: rocprofv3 --pmc / --kernel-trace wrap this)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jepsen_amd import _native, synth  # noqa: E402

n_keys = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cols, _ = synth.cas_register(n_keys=n_keys, ops_per_key=500, threads_per_key=10, readers=5, n_values=5,
                             process_limit=20, groups=10, init_nil=True, p_info=0.02, p_invalid=0.01,
                             nemesis_every=10000, seed=3)   # the bench.py C3 workload
ctx = _native.Context(0)
for _ in range(reps):
    v, s = ctx.check_cas_independent(cols)
print(f"keys={s.n_keys} invalid={s.n_invalid} unknown={s.n_unknown} explored={s.explored} "
      f"device_ms={s.device_ms:.2f} dfs_ms={s.dfs_ms:.2f}")
