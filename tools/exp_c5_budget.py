"""Experiment: C5-shaped keys at several budgets / phase-3 wave counts
(JH_DEBUG=1 prints the phase timings). usage: exp_c5_budget.py keys budget..."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jepsen_amd import _native, synth  # noqa: E402

n = int(sys.argv[1])
cols, _ = synth.cas_register(n_keys=n, ops_per_key=500, threads_per_key=50, readers=25,
                             process_limit=100, p_info=0.2, p_invalid=0.01, seed=5)
ctx = _native.Context(0)
for b in sys.argv[2:]:
    t = time.perf_counter()
    v, s = ctx.check_cas_independent(cols, budget=int(b))
    print(f"budget={b} keys={n} unknown={s.n_unknown} explored={s.explored} "
          f"device_ms={s.device_ms:.1f} wall={time.perf_counter() - t:.2f}s", flush=True)
