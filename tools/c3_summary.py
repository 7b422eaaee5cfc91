"""Summarise C3 bench lines of gpu_bfs_ab.sh logs (ms/step and phase times).
    python tools/c3_summary.py gpurun_out/bfsab/*.log"""
import json
import sys

for path in sys.argv[1:]:
    for ln in open(path):
        if ln.startswith("{"):
            d = json.loads(ln)
            c = d["config"]
            print(f"{path}: {d['ms_per_step']:.2f} ms/step | phase1 {c.get('phase1_ms', 0):.1f} "
                  f"seq {c.get('phase2_seq_ms', 0):.1f} bfs {c.get('phase2_bfs_ms', 0):.1f}")
