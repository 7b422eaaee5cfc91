"""HBM traffic per launch of a kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes (one counter per pass, MI355X_MICROARCH.md "HBM"), written as the JSON
that bench.py puts into its roofline object as `traffic`.

    python tools/pmc_traffic.py <pmc-dir> profiles/r02/traffic_<workload>_<kernel>.json <kernel-substring> <workload>

Both counters are in KiB. The guide's gfx950 calibration: FETCH_SIZE reports
1/2 of the bytes of wide (16 B/lane) coalesced streaming reads, WRITE_SIZE is
exact for 16 B/lane streaming stores; other access widths are uncalibrated.
The search kernel's reads are 8-16 B scattered loads (tables, memo probes,
stack refills) and its writes 8 B scattered stores (evictions, stack spills),
so the raw sum is reported (no x2), with the raw counters beside it.
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]) * 1024.0)
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_lin_seq<true>"
    workload = sys.argv[4] if len(sys.argv) > 4 else "c3"
    fetch, nf = per_launch(src, "FETCH_SIZE", kernel)
    write, nw = per_launch(src, "WRITE_SIZE", kernel)
    if fetch is None or write is None:
        sys.exit(f"no FETCH_SIZE/WRITE_SIZE rows for {kernel} under {src}")
    # the profiled run's own work (tools/run_once.py's last line): under --pmc
    # rocprofv3 serializes dispatches, so the phase-2 race runs differently
    # from the bench and the traffic is compared with the same run's
    # algorithmic bytes, not the bench's
    run = {}
    try:
        last = [ln for ln in open(os.path.join(src, "fetch.log")) if ln.startswith("keys=")][-1]
        run = {k: float(v) for k, v in (f.split("=") for f in last.split()) if k}
    except (OSError, IndexError, ValueError):
        pass
    alg = None
    if "seq_probes" in run and "k_lin_seq" in kernel:
        alg = 56.0 * run["deferred_entries"] + 16.0 * run["seq_probes"]  # per call (the last of the reps)
    out = {"kernel": kernel, "fetch_bytes": fetch, "write_bytes": write,
           "profiled_run": run, "alg_bytes_same_run": alg,
           "traffic_bytes": fetch + write, "launches": [nf, nw],
           "correction": "none: scattered 8-16 B accesses are uncalibrated on gfx950 (MI355X_MICROARCH.md HBM)",
           "workload": f"tools/run_once.py {workload} 2 (the bench.py {workload} rank-0 history)"}
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
