# lin + limits GPU tests, then the C3 rank-0 bench line (no CPU baselines).
O=${1:-gpurun_out/lin}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_limits.py tests/test_c_harness.py -x -v --timeout 300 --timeout-method thread > $O/lin_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 > $O/bench_r0.log 2>&1
