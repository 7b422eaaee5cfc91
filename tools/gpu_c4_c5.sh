# C5 (50 threads/key, p_info 0.2) and C4 (125k-key shard) bench lines, with parity vs the oracle
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
JH_DEBUG=1 timeout -k 10 400 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 500 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1
