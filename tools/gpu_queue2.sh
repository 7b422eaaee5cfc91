cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q2
timeout -k 10 400 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 200 --timeout-method thread > gpurun_out/q2/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_queue.py > gpurun_out/q2/bench.log 2>&1
