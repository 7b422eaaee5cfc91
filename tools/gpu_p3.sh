# parity tests (lin), then C3 / C5 / C4 bench lines with phase timings
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_lin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_lin.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-parity > gpurun_out/bench_c3.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c5.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/bench_c4.log 2>&1
