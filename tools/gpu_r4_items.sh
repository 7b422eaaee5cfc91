# Round 4: BFS round items per (configuration, 8 members) (HEAD) against one
# configuration per lane (JH_BFS_ITEMS=0, round 2's layout): C4, C3, ranks 3/6.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_items.sh <outdir>
O=${1:-gpurun_out/r4items}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
for rep in 1 2; do
  timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_head_$rep.json 2> $O/c4_head_$rep.err || exit 1
  JH_LIB=$V/libjh_items0.so timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_items0_$rep.json 2> $O/c4_items0_$rep.err || exit 1
done
for rk in 0 3 6; do
  timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_head.json 2> $O/c3r${rk}_head.err || exit 1
  JH_LIB=$V/libjh_items0.so timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_items0.json 2> $O/c3r${rk}_items0.err || exit 1
done
exit 0
