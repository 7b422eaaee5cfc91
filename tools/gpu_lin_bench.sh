# linearizability parity tests, then the bench with in-kernel accounting and the plain bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_lin.log 2>&1 && \
JH_DEBUG=2 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-parity > gpurun_out/bench_dbg.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.log 2>&1
