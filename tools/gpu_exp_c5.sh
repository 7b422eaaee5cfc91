cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
JH_DEBUG=1 timeout -k 10 300 python -u tools/exp_c5_budget.py 1000 262144 524288 1048576 > gpurun_out/exp_c5.log 2>&1 || exit 1
JH_P3_WAVES=370 JH_DEBUG=1 timeout -k 10 300 python -u tools/exp_c5_budget.py 1000 1048576 > gpurun_out/exp_c5_w370.log 2>&1
