# GPU parity tests, then the bench with in-kernel cycle accounting
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "not c2_scale" > gpurun_out/gpu_tests.log 2>&1 && \
JH_DEBUG=2 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-parity > gpurun_out/bench_dbg.log 2>&1
