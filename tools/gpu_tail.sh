# counter/set parity (new pairing kernel), lin parity with tail deferral on, C3 phase timings A/B over JH_TAIL_DEFER
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_counter_set.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_cs.log 2>&1 || exit 1
JH_TAIL_DEFER=1024 timeout -k 10 900 python -u -m pytest tests/test_gpu_lin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_lin_tail.log 2>&1 || exit 1
for t in 0 1024 2048 3072; do
  JH_TAIL_DEFER=$t JH_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 > gpurun_out/tail_$t.log 2>&1 || exit 1
done
