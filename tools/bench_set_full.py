"""checker/set-full measurement (jepsen/src/jepsen/checker.clj:236-534)
on one MI355X: 1 M distinct adds by 20 processes, a whole-set read every 250
rounds of adds (200 reads, ~100 M read elements), 300 lost and 1 000 stale
elements (jepsen_amd/synth.py set_full_history, seed 6).

One JSON line. The history is resident in HBM before the timed region; a
step is one jh_check_set_full call including the D2H of its element lists.
`roofline`: algorithmic bytes (56 B per entry + 8 B per read element, read
once, + 8 B per listed element) over the call's time, against 8 TB/s; the
per-kernel split is in the rocprofv3 --stats summary (profiles/).
`cpu_baseline`: oracle/set_full_np.py (numpy, vectorised over elements, one
core) on the same history; `parity_vs_oracle` compares every list, count,
quantile and worst-stale entry with it.

    python tools/bench_set_full.py [--adds 1000000] [--steps 5] [--warmup 1] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_c2 import DevCols, timed, PEAK_HBM_GBS   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--adds", type=int, default=1_000_000)
    ap.add_argument("--read-every", type=int, default=250)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from jepsen_amd import _native, checker, synth
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    t0 = time.perf_counter()
    cols, tcol = synth.set_full_history(n_adds=args.adds, n_procs=20, read_every=args.read_every,
                                        n_lost=300, n_stale=1000, seed=6)
    gen_s = time.perf_counter() - t0
    d = DevCols(cols, dev)
    dt = torch.from_numpy(tcol).to(dev)
    r, sec = timed(lambda: ctx.check_set_full(d, dt.data_ptr(), on_device=True, list_cap=1 << 21),
                   args.steps, args.warmup)
    n, naux = int(cols.n), int(len(cols.aux))
    listed = r["lost_count"] + r["never_read_count"] + r["stale_count"]
    alg = 56.0 * n + 8.0 * naux + 8.0 * listed
    cpu, parity = None, None
    if not args.no_cpu:
        from oracle import set_full_np as SN
        t0 = time.perf_counter()
        want = SN.set_full_cols(cols, tcol)
        ct = time.perf_counter() - t0
        got = checker.set_full_result(r, cols, tcol)
        got["worst-stale"] = [(w["element"], w["stable-latency"], w["known"]["index"],
                               w["last-absent"]["index"] if w["last-absent"] else -1)
                              for w in got["worst-stale"]]
        parity = got == want
        cpu = {"value": n / ct, "unit": "entries/s", "cores": 1, "kind": "port",
               "sample": f"the whole history ({n} entries, {naux} read elements), "
                         f"oracle/set_full_np.py ({ct:.2f} s)"}
    print(json.dumps({
        "metric": "history entries verified/sec, checker/set-full", "value": n / sec,
        "unit": "entries/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": sec * 1e3, "higher_is_better": True, "dtype": "int64",
        "data": "synthetic (jepsen_amd/synth.py set_full_history, seed 6)",
        "config": {"workload": "set-full: 1M adds, whole-set reads", "entries": n, "adds": args.adds,
                   "reads": r["n_reads"], "read_elements": naux, "lost": r["lost_count"],
                   "stale": r["stale_count"], "never_read": r["never_read_count"],
                   "valid": r["valid"], "device_ms": r["device_ms"], "gen_s": round(gen_s, 1)},
        "roofline": {"bound": "hbm", "kernel": "whole jh_check_set_full call",
                     "achieved": alg / sec / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": alg / sec / 1e9 / PEAK_HBM_GBS, "traffic": None},
        "cpu_baseline": cpu, "parity_vs_oracle": parity}))


if __name__ == "__main__":
    main()
