# A/B: parity tests, then phase timings of the C3 bench for each library variant given as argument
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_lin.log 2>&1 || exit 1
for v in "$@"; do
  lib=jepsen_amd/libjh.so; [ "$v" != base ] && lib=jepsen_amd/variants/libjh_$v.so
  JH_QUICK_BUDGET=${QB:-16384} JH_LIB=$lib JH_DEBUG=2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-parity > gpurun_out/ab/$v.log 2>&1 || exit 1
done
