# lin GPU tests, bench (rank 0 with CPU baseline), rehearsal of ranks 3 and 6
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p2
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/p2/tests.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/p2/bench_r0.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --seed-rank 3 > gpurun_out/p2/bench_r3.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --seed-rank 6 > gpurun_out/p2/bench_r6.log 2>&1
