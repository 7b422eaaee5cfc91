# every GPU test + smoke at HEAD (the in-tree .so the round-end run loads)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/head2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/head2/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/head2/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/head2/bench.log 2>&1
