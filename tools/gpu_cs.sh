# counter/set parity tests, then the C2 bench + kernel profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_counter_set.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_cs.log 2>&1 || exit 1
bash tools/gpu_c2.sh
