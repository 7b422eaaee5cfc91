"""Summarise the C5 bench lines (and [jh-xw-prof] lines) of gpu_xw.sh logs.
    python tools/c5_summary.py gpurun_out/xw2/*.log"""
import json
import sys

for path in sys.argv[1:]:
    for ln in open(path):
        if ln.startswith("{"):
            d = json.loads(ln)
            ph = d["config"]["phases"]
            print(f"{path}: {d['ms_per_step']:.1f} ms/step | xw {ph['xw']['ms']:.1f} bfs {ph['bfs']['ms']:.1f} "
                  f"wide {ph['wide']['ms']:.1f} | xw probes {ph['xw']['probes']:.0f} unknown {d['config']['unknown_keys']}")
        elif "xw-prof" in ln:
            print(f"{path}: {ln.strip()}")
