# BFS iteration: lin parity tests, then per-rank timing (bench.py --seed-rank)
# and the per-workgroup BFS accounting of ranks 3 and 6.
#   gpurun -- bash tools/gpu_bfs_iter.sh <outdir>
O=${1:-gpurun_out/bfsiter}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > $O/lin_tests.log 2>&1 || exit 1
for RK in 0 3 6; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --seed-rank $RK > $O/bench_r$RK.log 2>&1 || exit 1
  JH_DEBUG=2 timeout -k 10 120 python -u tools/run_once.py c3 1 $RK > $O/dbg_r$RK.log 2>&1 || exit 1
done
