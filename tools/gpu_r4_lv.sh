# Round 4: the count pass's same-layer liveness, one node per thread (HEAD)
# against one item per (node, 8 members) (JH_BFS_LV_ITEMS=1, round 3):
# C3 ranks 0/3/4/6, C4; the lin tests.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_lv.sh <outdir>
O=${1:-gpurun_out/r4lv}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lin.py > $O/lin_tests.log 2>&1 || exit 1
for rk in 0 3 4 6; do
  timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_head.json 2> $O/c3r${rk}_head.err || exit 1
  JH_LIB=$V/libjh_lv1.so timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_lv1.json 2> $O/c3r${rk}_lv1.err || exit 1
done
timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_head.json 2> $O/c4_head.err || exit 1
JH_LIB=$V/libjh_lv1.so timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_lv1.json 2> $O/c4_lv1.err || exit 1
exit 0
