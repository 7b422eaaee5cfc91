# C5 line and rank-3 rehearsal after the phase-3 condition on the budget extension
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5b
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5b/tests.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --steps 3 --warmup 1 --seed-rank 3 > gpurun_out/c5b/bench_r3.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 500 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/c5b/bench_c5.log 2>&1
