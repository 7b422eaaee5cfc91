# linearizability GPU parity tests, then C3 phase timings at two quick budgets
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qab
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_lin.log 2>&1 || exit 1
for qb in "$@"; do
  JH_QUICK_BUDGET=$qb JH_DEBUG=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/qab/q$qb.log 2>&1 || exit 1
done
