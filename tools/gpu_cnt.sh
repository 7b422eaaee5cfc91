# counter/set parity tests, then the C2 bench lines and kernel summary
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/c2
timeout -k 10 600 python -u -m pytest tests/test_gpu_counter_set.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_cs.log 2>&1 || exit 1
bash tools/gpu_c2.sh
