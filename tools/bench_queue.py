"""checker/total-queue and checker/queue (model/unordered-queue) measurement
(jepsen/src/jepsen/checker.clj:160-180, 536-628) on one MI355X: a
synthetic queue history of 4 M consecutive-integer enqueues (gen/queue,
generator.clj:405-416; ~9 M entries; jepsen_amd/synth.py queue_history, seed 8) with lost, unexpected and duplicated elements and a
final drain.

One JSON line per checker. The history is resident in HBM before the timed
region; a step is one jh_check_total_queue / jh_check_queue call including
the D2H of its multisets. `roofline`: algorithmic bytes (56 B per entry and
8 B per drained element read once, + 16 B per output pair) over the call's
time against 8 TB/s. `cpu_baseline`: oracle/queue.py (Python Counter, one
core) on the same history; `parity_vs_oracle` compares every count and
multiset (total-queue) and the verdict and failing row (queue).

    python tools/bench_queue.py [--enqueues 4000000] [--steps 5] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_c2 import DevCols, timed, PEAK_HBM_GBS   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--enqueues", type=int, default=4_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from jepsen_amd import _native, synth
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    cols = synth.queue_history(n_enqueues=args.enqueues, n_procs=10, n_lost=1000, n_unexpected=100,
                               n_duplicated=100, n_repeat=1000, drain_parts=10, seed=8)
    d = DevCols(cols, dev)
    n, naux = int(cols.n), int(len(cols.aux))
    ops = synth.queue_columns_to_ops(cols) if not args.no_cpu else None
    from oracle import queue as Q
    for name, call in (("total-queue", lambda: ctx.check_total_queue(d, pairs_cap=1 << 20, on_device=True)),
                       ("queue", lambda: ctx.check_queue(d, pairs_cap=1 << 23, on_device=True))):
        r, sec = timed(call, args.steps, args.warmup)
        alg = 56.0 * n + 8.0 * naux + 16.0 * sum(r["n_pairs"])
        cpu, parity = None, None
        if ops is not None:
            t0 = time.perf_counter()
            want = Q.total_queue(ops) if name == "total-queue" else Q.queue(ops)
            ct = time.perf_counter() - t0
            if name == "total-queue":
                parity = all(int(r[k + "_count"]) == want[k + "-count"] for k in
                             ("attempt", "acknowledged", "ok", "unexpected", "duplicated", "lost", "recovered"))
                for k in ("lost", "unexpected", "duplicated", "recovered"):
                    parity = parity and {int(v): int(c) for v, c in r[k]} == dict(want[k])
            else:
                parity = (r["valid"] == 0) == want["valid?"] and \
                    (want["valid?"] or r["fail_entry"] == want["fail-index"])
            cpu = {"value": n / ct, "unit": "entries/s", "cores": 1, "kind": "port",
                   "sample": f"the whole history ({n} entries), oracle/queue.py ({ct:.2f} s)"}
        print(json.dumps({
            "metric": f"history entries verified/sec, checker/{name}", "value": n / sec,
            "unit": "entries/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": sec * 1e3, "higher_is_better": True, "dtype": "int64",
            "data": "synthetic (jepsen_amd/synth.py queue_history, seed 8)",
            "config": {"workload": f"{name}: 4M enqueues", "entries": n, "drained": naux,
                       "valid": r["valid"], "n_pairs": r["n_pairs"], "device_ms": r["device_ms"]},
            "roofline": {"bound": "hbm", "kernel": f"whole jh_check_{name.replace('-', '_')} call",
                         "achieved": alg / sec / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": alg / sec / 1e9 / PEAK_HBM_GBS, "traffic": None},
            "cpu_baseline": cpu, "parity_vs_oracle": parity}), flush=True)


if __name__ == "__main__":
    main()
