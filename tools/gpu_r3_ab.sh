# Round 3 A/B of jh_lin_opts knobs on C3 ranks 0 / 3 / 6 (bench.py --opt):
#   gpurun --timeout 1200 -- bash tools/gpu_r3_ab.sh <outdir> "<opt set>" ["<opt set>" ...]
# an opt set is space-separated FIELD=INT pairs, "-" for the defaults; one
# line per (set, rank) in <outdir>/ab.txt
O=${1:-gpurun_out/ab}
shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for set in "$@"; do
  args=""
  if [ "$set" != "-" ]; then for kv in $set; do args="$args --opt $kv"; done; fi
  for rank in 0 3 6; do
    f=$O/ab_$(echo "$set" | tr ' =' '_-')_r$rank.log
    timeout -k 10 150 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank $rank $args > $f 2>&1 || exit 1
    python - "$f" "$set" "$rank" >> $O/ab.txt <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
c = d["config"]
print(f"opts={sys.argv[2]!r:28} rank={sys.argv[3]} ms={d['ms_per_step']:.2f} phase1={c['phase1_ms']:.2f} "
      f"seq={c['phase2_seq_ms']:.2f} bfs={c['phase2_bfs_ms']:.2f} deferred={c['deferred_keys']}")
EOF
  done
done
cat $O/ab.txt
