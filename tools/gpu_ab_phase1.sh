cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab1
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_limits.py tests/test_c_harness.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab1/lin.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --e2e 0 > gpurun_out/ab1/bench_default.log 2>&1 || exit 1
for V in ${VARIANTS:-q7 q7b}; do
  JH_LIB=$GRAFT_REPO_ROOT/jepsen_amd/variants/libjh_$V.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --e2e 0 > gpurun_out/ab1/bench_$V.log 2>&1 || exit 1
done
