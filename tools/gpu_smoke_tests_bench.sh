cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "not c2_scale" > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.log 2>&1
