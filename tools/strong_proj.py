"""Projected strong scaling of the north_star's own configuration (VERDICT r5
item 3): ONE 10k-key C3 history split by key over N GPUs (bench.py --workload
c3s --shard r/N, each shard rehearsed on one GPU). A step on N GPUs ends
with its slowest shard, so the projection is the max over the shards of
ms_per_step; entries/s = the whole history's entries / that time.

    python tools/strong_proj.py <dir with c3s_<r>of<N>.json> [one-GPU line json]
"""
import glob
import json
import os
import re
import sys

d = sys.argv[1]
lines = {}
for f in glob.glob(os.path.join(d, "c3s_*of*.json")):
    m = re.search(r"c3s_(\d+)of(\d+)\.json$", f)
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    lines.setdefault(int(m.group(2)), {})[int(m.group(1))] = j
out = {}
one = None
if len(sys.argv) > 2:
    one = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    out[1] = {"ms": one["ms_per_step"], "entries_per_s": one["value"]}
for n, by in sorted(lines.items()):
    if len(by) != n:
        continue
    ms = {r: j["ms_per_step"] for r, j in by.items()}
    glob_entries = next(iter(by.values()))["shard"]["global_entries"]
    worst = max(ms, key=ms.get)
    out[n] = {"ms": ms[worst], "slowest_shard": worst, "shard_ms": [round(ms[r], 2) for r in sorted(ms)],
              "entries_per_s": glob_entries / (ms[worst] / 1e3),
              "speedup_vs_1": (out[1]["ms"] / ms[worst]) if 1 in out else None}
print(json.dumps(out, indent=1))
