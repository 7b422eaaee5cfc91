"""HBM traffic per launch of a kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes (one counter per pass, MI355X_MICROARCH.md "HBM") over one history,
written as the JSON bench.py puts into its roofline object (`traffic`,
`traffic_over_alg_same_run`).

    python tools/pmc_traffic.py <pmc-dir> <kernel-substring> <workload> <seed> [bench-label]

-> profiles/r06/traffic_<workload>_s<seed>_<kernel>.json (bench.traffic_name).
Both counters are in KiB. The guide's gfx950 calibration: FETCH_SIZE reports
1/2 of the bytes of wide (16 B/lane) coalesced streaming reads, WRITE_SIZE is
exact for 16 B/lane streaming stores; other access widths are uncalibrated.
The search kernels' reads are 8-16 B scattered loads (tables, memo probes,
stack refills) and their writes 8-16 B scattered stores (evictions, stack
spills), so the raw sum is reported (no x2), with the raw counters beside it.
The algorithmic bytes are the profiled run's own (tools/run_once.py prints its
jh_summary), so the ratio compares traffic and work of the same run.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import PHASES, TRAFFIC_DIR, phase_alg_bytes, traffic_name  # noqa: E402


def per_launch(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    src, kernel, workload, seed = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    # the bench.PHASES label the file is keyed by, when the rocprof name
    # carries more template arguments (k_lin_seq_lw<false, MemoCfg<10, 17> >)
    label = sys.argv[5] if len(sys.argv) > 5 else kernel
    fetch, write = per_launch(src, "FETCH_SIZE", kernel), per_launch(src, "WRITE_SIZE", kernel)
    if not fetch or not write:
        sys.exit(f"no FETCH_SIZE/WRITE_SIZE rows for {kernel} under {src}")
    run = {}
    for log in ("fetch.log", "write.log"):
        try:
            lines = [ln for ln in open(os.path.join(src, log)) if ln.startswith("SUMMARY ")]
            run[log] = json.loads(lines[-1][8:])
        except (OSError, IndexError, ValueError):
            pass
    # the phase whose kernel this is (bench.PHASES): its entries and probes in each pass's run
    alg, ents, probes, ms = {}, [], [], []
    for log, d in run.items():
        for name, (tf, pf, ef, kf, kern) in PHASES.items():
            if kern.split("<")[0] in label and (("<" not in label) or kern in label) and d.get(tf, 0) > 0:
                ent = d["entries"] if ef is None else d[ef]
                alg[log] = phase_alg_bytes(name, d, d["entries"])
                ents.append(ent); probes.append(d[pf]); ms.append(d[tf])
                break
    # every launch of the kernel in a pass (reps calls) counts; per launch = mean
    f1, w1 = sum(fetch) / len(fetch), sum(write) / len(write)
    a = [alg[k] for k in ("fetch.log", "write.log") if k in alg]
    alg_run = sum(a) / len(a) if a else None
    out = {"kernel": label, "rocprof_kernel_match": kernel, "workload": workload, "seed": seed,
           "fetch_bytes": f1, "write_bytes": w1, "traffic_bytes": f1 + w1,
           "launches": [len(fetch), len(write)], "alg_bytes_same_run": alg_run,
           "traffic_over_alg": (f1 + w1) / alg_run if alg_run else None,
           # the serialized --pmc run's own phase (bench.py scales by algorithmic bytes)
           "pmc_entries": sum(ents) / len(ents) if ents else 0.0,
           "pmc_probes": sum(probes) / len(probes) if probes else 0.0,
           "pmc_phase_ms": sum(ms) / len(ms) if ms else 0.0,
           "schedule": "serialized: rocprofv3 --pmc runs one kernel at a time",
           "profiled_runs": run,
           "correction": "none: scattered 8-16 B accesses are uncalibrated on gfx950 (MI355X_MICROARCH.md HBM)"}
    dst = os.path.join(TRAFFIC_DIR, traffic_name(workload, seed, label))
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "profiled_runs"}))


if __name__ == "__main__":
    main()
