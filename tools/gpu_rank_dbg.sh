# per-wave DFS accounting (JH_DEBUG=2) on rank 6's history, and ranks 4 and 7 lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rk
JH_DEBUG=2 timeout -k 10 300 python -u bench.py --no-cpu --no-parity --steps 2 --warmup 1 --seed-rank 6 > gpurun_out/rk/r6_dbg.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --seed-rank 4 > gpurun_out/rk/r4.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --seed-rank 7 > gpurun_out/rk/r7.log 2>&1
