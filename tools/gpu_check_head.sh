# HEAD check: GPU tests, smoke, default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/head
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/head/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/head/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/head/bench.log 2>&1
