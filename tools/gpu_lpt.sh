# LPT order of the phase-1 list: lin GPU tests, C3 bench A/B, rank-6 rehearsal
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lpt
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lpt/tests.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 > gpurun_out/lpt/bench_r0.log 2>&1 || exit 1
JH_NO_LPT=1 JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-parity --e2e 0 > gpurun_out/lpt/bench_r0_nolpt.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --steps 3 --warmup 1 --seed-rank 6 > gpurun_out/lpt/bench_r6.log 2>&1
