# A/B of the phase-1 quick budget: phase timings of the C3 bench per value
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qab
for qb in "$@"; do
  JH_QUICK_BUDGET=$qb JH_DEBUG=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/qab/q$qb.log 2>&1 || exit 1
done
