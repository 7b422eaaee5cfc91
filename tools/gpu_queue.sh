# queue checkers + set-full: GPU parity tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q
timeout -k 10 500 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_set_full.py -x -v --timeout 200 --timeout-method thread > gpurun_out/q/tests.log 2>&1
