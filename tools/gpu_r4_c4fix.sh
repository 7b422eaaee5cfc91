# Round 4: the BFS set's per-insert reservation near the limit (C4 phase 2),
# C4 / C3 / ranks 3 and 6, and the lin tests.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_c4fix.sh <outdir>
O=${1:-gpurun_out/r4c4fix}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_head.json 2> $O/c4_head.err || exit 1
timeout -k 10 120 $B --steps 5 --warmup 1 > $O/c3_head.json 2> $O/c3_head.err || exit 1
for rk in 3 6; do timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_head.json 2> $O/c3r${rk}_head.err || exit 1; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lin.py tests/test_gpu_limits.py > $O/lin_tests.log 2>&1 || exit 1
exit 0
