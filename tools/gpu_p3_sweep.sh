# phase-3 concurrency sweep on C5-shaped keys
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in 1024 256 64; do
  JH_P3_WAVES=$w JH_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c5 --keys 300 --steps 1 --warmup 0 --no-cpu --no-parity --e2e 0 > gpurun_out/p3w_$w.log 2>&1 || exit 1
done
