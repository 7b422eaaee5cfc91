"""Host-buffer calls timed (jh_ingest.hip A/B): C3 cas-independent and the
100 M-entry C2 counter, three calls each, from numpy (pageable) columns.
    JH_LIB=... [JH_INGEST_PLAIN=1] [JH_INGEST_TRACE=1] python tools/ingest_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _native, synth  # noqa: E402

ctx = _native.Context(0)
out = {}
wl = WORKLOADS["c3"]
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"], **wl["gen"])
ts = []
for _ in range(4):
    t0 = time.perf_counter()
    ctx.check_cas_independent(cols, budget=wl.get("budget"), exact_count=False)
    ts.append((time.perf_counter() - t0) * 1e3)
out["c3_ms"] = ts
del cols
cols = synth.counter(n_ops=50_000_000, n_procs=10, read_every=101, p_fail=0.05, p_info=0.01, n_bad_reads=10, seed=2)
ts = []
for _ in range(4):
    t0 = time.perf_counter()
    ctx.check_counter(cols, reads_cap=1 << 20)
    ts.append((time.perf_counter() - t0) * 1e3)
out["c2_counter_ms"] = ts
print(json.dumps(out), flush=True)
