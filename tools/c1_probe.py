"""One C1 stale-read key (test_gpu_configs.py::test_c1_variants) through
jh_check_cas with given jh_lin_opts flags, timed: python tools/c1_probe.py <seed> <flags>"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from jepsen_amd import _native, synth  # noqa: E402

seed, flags = int(sys.argv[1]), int(sys.argv[2])
cols, _ = synth.cas_register(n_keys=1, ops_per_key=5000, threads_per_key=5, readers=2, groups=1, p_info=0.01,
                             seed=seed, keyed=False, init_nil=True, process_limit=10 ** 6, p_invalid=1.0)
ctx = _native.Context(0)
t0 = time.perf_counter()
v = ctx.check_cas(cols, budget=1 << 24, flags=flags)
print(json.dumps({"seed": seed, "flags": flags, "s": round(time.perf_counter() - t0, 3), "verdict": list(map(int, v))}),
      flush=True)
