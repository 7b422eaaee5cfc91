# Phase-2 late helpers (k_lin_wg in helper mode): lin parity tests, the C3 bench
# line with and without helpers, and the rank-3/4/6 rehearsals, one gpurun call.
#   gpurun -- bash tools/gpu_helpers.sh <outdir>
O=${1:-gpurun_out/help}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > $O/lin_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 > $O/bench_r0.log 2>&1 || exit 1
JH_HELPERS=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 > $O/bench_r0_nohelp.log 2>&1 || exit 1
for RK in 3 4 6; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --seed-rank $RK > $O/bench_r$RK.log 2>&1 || exit 1
done
