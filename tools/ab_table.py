"""Table of an A/B directory of bench lines (<name>_r<rank>_<rep>.json):
ms per step per variant and rank, and spec counters.
    python tools/ab_table.py <dir>"""
import collections
import glob
import json
import os
import re
import sys

d = sys.argv[1]
t = collections.defaultdict(lambda: collections.defaultdict(list))
sp = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*_r*_*.json"))):
    m = re.match(r"(.+)_r(\d+)_(\d+)\.json$", os.path.basename(f))
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    t[m.group(1)][int(m.group(2))].append(j["ms_per_step"])
    sp[m.group(1)].append((j["config"].get("spec") or {}).get("merges", 0))
ranks = sorted({r for v in t.values() for r in v})
print("variant".ljust(14) + "".join(f"r{r}".rjust(22) for r in ranks) + "   merges")
for v in sorted(t):
    print(v.ljust(14) + "".join(("/".join(f"{x:.1f}" for x in t[v][r]) + f" ({sum(t[v][r]) / len(t[v][r]):.1f})").rjust(22)
                                if t[v][r] else "".rjust(22) for r in ranks) + f"   {sp[v]}")
