# phase-1 tail cut: lin GPU tests, C3 bench (A/B), rank-6 rehearsal, C5 line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tc
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tc/tests.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 > gpurun_out/tc/bench_r0.log 2>&1 || exit 1
JH_NO_TAIL_CUT=1 JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-parity --e2e 0 > gpurun_out/tc/bench_r0_nocut.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --steps 3 --warmup 1 --seed-rank 6 > gpurun_out/tc/bench_r6.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 500 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/tc/bench_c5.log 2>&1
