# phase timings + rocprofv3 kernel stats of the bench, then the C2 counter scale test
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export JH_DEBUG=1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/bench2.log 2>&1 && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-parity > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1) && \
timeout -k 10 600 python -m pytest tests/test_gpu_counter_set.py -x -q -k c2_scale > gpurun_out/c2.log 2>&1
