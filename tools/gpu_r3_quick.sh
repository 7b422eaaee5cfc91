# Round 3: lin + counter/set parity tests, C3 / C5 / C2 bench lines after a change.
#   gpurun --timeout 1200 -- bash tools/gpu_r3_quick.sh <outdir>
O=${1:-gpurun_out/r3q}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_counter_set.py -x -v --timeout 200 --timeout-method thread > $O/cs_tests.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_limits.py -x -v --timeout 300 --timeout-method thread > $O/lin_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_c2.py --no-cpu > $O/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu --e2e 0 > $O/bench_c5.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --seed-rank 3 > $O/bench_c3_rank3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --seed-rank 6 > $O/bench_c3_rank6.log 2>&1 || exit 1
JH_LIB=$R/jepsen_amd/variants/libjh_tune.so JH_DEBUG=2 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank 3 > $O/dbg_rank3.log 2>&1 || exit 1
JH_LIB=$R/jepsen_amd/variants/libjh_tune.so JH_DEBUG=1 JH_DEFER_TIMES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/dbg_rank0.log 2>&1 || exit 1
JH_LIB=$R/jepsen_amd/variants/libjh_stats.so JH_DEBUG=2 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/stats_rank0.log 2>&1 || exit 1
exit 0
