# Round 4: late helpers take keys in the deferral order (least phase-1
# progress first, JH_HELP_BY_ORDER=1) against the longest-running key (HEAD):
# C3 ranks 0-7 alternating, C4; timelines of rank 0 for both.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_help.sh <outdir>
O=${1:-gpurun_out/r4help}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
for rk in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_head.json 2> $O/c3r${rk}_head.err || exit 1
  JH_LIB=$V/libjh_hord.so timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_hord.json 2> $O/c3r${rk}_hord.err || exit 1
done
timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_head.json 2> $O/c4_head.err || exit 1
JH_LIB=$V/libjh_hord.so timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_hord.json 2> $O/c4_hord.err || exit 1
JH_LIB=$V/libjh_tune.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_head.json 2> $O/tl_head.err || exit 1
JH_LIB=$V/libjh_hordt.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_hord.json 2> $O/tl_hord.err || exit 1
exit 0
