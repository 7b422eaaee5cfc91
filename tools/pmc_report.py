"""Per-DFS-step view of the PMC passes written by tools/gpu_pmc.sh."""
import csv
import glob
import os
import sys

root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "pmc")
steps = float(sys.argv[1]) if len(sys.argv) > 1 else 47429888.0
for v in sorted(os.listdir(root)):
    d = {}
    for f in glob.glob(os.path.join(root, v, "p*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("::")[1].split("(")[0]
            d.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in sorted(d.items()):
        if "dfs" not in k:
            continue
        per = {n: c[n] / steps for n in c}
        print(f"{v:10s} {k:22s} " + " ".join(f"{n.replace('SQ_', '')}={per[n]:.1f}" for n in sorted(per) if n != "SQ_WAVES"))
