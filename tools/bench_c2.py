"""C2 measurement (BASELINE.json configs[1]): checker/counter and checker/set on
synthetic 100M-entry histories on one MI355X.

Prints one JSON line per checker. The history is resident in HBM before the
timed region (columns copied once); a step is one jh_check_counter /
jh_check_set call, including its D2H of the result (the :reads triples or the
run-length sets). `roofline` is whole-call algorithmic bytes (SURVEY 8(d):
56 B per entry read once, +24 B per :reads triple, +16 B per run of the four
result sets; the set's bitmaps 16 B per word of the four) over the call's
time, against the 8 TB/s HBM peak; the
per-kernel split is in the rocprofv3 --stats summary (profiles/).

    python tools/bench_c2.py [--entries 100000000] [--steps 5] [--warmup 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PEAK_HBM_GBS = 8000.0


class DevCols:
    """Device-resident columns (torch tensors kept alive) in the include/jh.h layout."""

    def __init__(self, cols, dev):
        import torch
        self._t = {}
        for k in ("process", "type", "f", "key", "value", "value2"):
            self._t[k] = torch.from_numpy(np.ascontiguousarray(getattr(cols, k))).to(dev)
            setattr(self, k, self._t[k].data_ptr())
        aux = getattr(cols, "aux", None)
        if aux is not None and len(aux):
            self._t["aux"] = torch.from_numpy(np.ascontiguousarray(aux)).to(dev)
            self.aux, self.n_aux = self._t["aux"].data_ptr(), len(aux)
        else:
            self.aux, self.n_aux = 0, 0
        self.n, self.n_keys = int(cols.n), int(cols.n_keys)


def timed(fn, steps, warmup):
    import torch
    for _ in range(warmup):
        r = fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entries", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=10_000_000,
                    help="entries of the same generator timed on the CPU oracle")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--e2e", action="store_true",
                    help="also time calls on host buffers (H2D of the columns included)")
    args = ap.parse_args()
    import torch
    from jepsen_amd import _native, synth
    from oracle import oracle
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    lines = []

    # ---- counter: add:read = 100:1, add 1, p_fail 5%, p_info 1%, 10 bad reads
    half = args.entries // 2
    cols = synth.counter(n_ops=half, n_procs=10, read_every=101, p_fail=0.05, p_info=0.01,
                         n_bad_reads=10, seed=2)
    d = DevCols(cols, dev)
    # the triples land in a reused page-locked buffer (jh_host_alloc), as a
    # JNA shim would keep one per checker
    reads_buf = _native.HostBuffer(3 << 20, np.int64)
    r, sec = timed(lambda: ctx.check_counter(d, reads_cap=1 << 20, on_device=True, out=reads_buf.array),
                   args.steps, args.warmup)
    n = int(cols.n)
    alg = 56.0 * n + 24.0 * r["n_reads"]
    e2e = None
    if args.e2e:
        _, hs = timed(lambda: ctx.check_counter(cols, reads_cap=1 << 20, out=reads_buf.array), 2, 1)
        e2e = {"ms_per_call": hs * 1e3, "entries_per_s": n / hs}
    cpu = None
    if not args.no_cpu:
        cs = synth.counter(n_ops=args.cpu_sample // 2, n_procs=10, read_every=101, p_fail=0.05,
                           p_info=0.01, n_bad_reads=10, seed=2)
        t0 = time.perf_counter()
        oracle.check_counter(cs)
        ct = time.perf_counter() - t0
        cpu = {"value": cs.n / ct, "unit": "entries/s", "cores": 1, "kind": "port",
               "sample": f"{int(cs.n)} entries of the same generator, oracle/jh_oracle.c counter on one core "
                         f"(the reference's loop is one sequential pass, checker.clj:698-734) ({ct:.2f} s)"}
    lines.append({"metric": "history entries verified/sec, checker/counter (C2)", "value": n / sec,
                  "unit": "entries/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
                  "ms_per_step": sec * 1e3, "higher_is_better": True, "dtype": "int64",
                  "data": "synthetic (jepsen_amd/csrc/gen.cpp counter, seed 2)",
                  "config": {"workload": "C2 counter", "entries": n, "reads": r["n_reads"],
                             "errors": r["n_errors"], "valid": r["valid"], "e2e_host_buffers": e2e},
                  "roofline": {"bound": "hbm", "kernel": "whole jh_check_counter call",
                               "achieved": alg / sec / 1e9, "peak": PEAK_HBM_GBS,
                               "unit": "GB/s", "frac": alg / sec / 1e9 / PEAK_HBM_GBS,
                               "traffic": None},
                  "cpu_baseline": cpu})
    del d, cols
    torch.cuda.empty_cache()

    # ---- set: distinct adds, p_fail 5%, p_info 2%, 100 lost, 10 unexpected
    cols = synth.set_history(n_adds=half, n_procs=10, p_fail=0.05, p_info=0.02, n_lost=100,
                             n_unexpected=10, seed=2)
    d = DevCols(cols, dev)
    # the product path: the four result sets come back as bitmaps (4 B per 32
    # elements of span); the runs output (16 B per run) is timed beside it
    bit_bufs = [_native.HostBuffer(1 << 22, np.uint32) for _ in range(4)]
    r, sec = timed(lambda: ctx.check_set_bitmaps(d, words_cap=1 << 22, on_device=True,
                                                 out=[b.array for b in bit_bufs]), args.steps, args.warmup)
    _, sec_runs = timed(lambda: ctx.check_set(d, runs_cap=1 << 25, on_device=True), 2, 1)
    n = int(cols.n)
    alg = 56.0 * n + 8.0 * d.n_aux + 16.0 * r["n_words"]
    e2e = None
    if args.e2e:
        _, hs = timed(lambda: ctx.check_set_bitmaps(cols, words_cap=1 << 22, out=[b.array for b in bit_bufs]), 2, 1)
        e2e = {"ms_per_call": hs * 1e3, "entries_per_s": n / hs}
    cpu = None
    if not args.no_cpu:
        cs = synth.set_history(n_adds=args.cpu_sample // 2, n_procs=10, p_fail=0.05, p_info=0.02,
                               n_lost=100, n_unexpected=10, seed=2)
        t0 = time.perf_counter()
        oracle.check_set(cs)
        ct = time.perf_counter() - t0
        cpu = {"value": cs.n / ct, "unit": "entries/s", "cores": 1, "kind": "port",
               "sample": f"{int(cs.n)} entries of the same generator, oracle/jh_oracle.c set on one core "
                         f"(the reference folds the history sequentially, checker.clj:182-234) ({ct:.2f} s)"}
    lines.append({"metric": "history entries verified/sec, checker/set (C2)", "value": n / sec,
                  "unit": "entries/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
                  "ms_per_step": sec * 1e3, "higher_is_better": True, "dtype": "int64",
                  "data": "synthetic (jepsen_amd/csrc/gen.cpp set, seed 2)",
                  "config": {"workload": "C2 set", "entries": n, "final_read": d.n_aux,
                             "lost": r["lost_count"], "unexpected": r["unexpected_count"],
                             "valid": r["valid"], "n_runs": r["n_runs"], "bitmap_words": r["n_words"],
                             "output": "jh_check_set_bitmaps (4 result bitmaps)",
                             "ms_per_call_runs_output": sec_runs * 1e3, "e2e_host_buffers": e2e},
                  "roofline": {"bound": "hbm", "kernel": "whole jh_check_set_bitmaps call",
                               "achieved": alg / sec / 1e9, "peak": PEAK_HBM_GBS,
                               "unit": "GB/s", "frac": alg / sec / 1e9 / PEAK_HBM_GBS,
                               "traffic": None},
                  "cpu_baseline": cpu})
    for ln in lines:
        print(json.dumps(ln))


if __name__ == "__main__":
    main()
