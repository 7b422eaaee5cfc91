# phase-1 quick budget sweep on the C3 bench (rank-0 history)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qs
for q in 4096 2048 1024 512; do
  JH_QUICK_BUDGET=$q JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-parity --e2e 0 --steps 5 --warmup 1 > gpurun_out/qs/q$q.log 2>&1 || exit 1
done
