# BFS exact counts for valid keys: heavy keys one by one, lin parity tests,
# the C3 bench line and the rank-3/4/6 rehearsals, one gpurun call.
O=${1:-gpurun_out/bfsc}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
JH_WG=0 timeout -k 10 200 python -u tools/heavy_keys.py > $O/hk.log 2>&1 || exit 1
JH_DEBUG=2 JH_WG=0 timeout -k 10 100 python -u tools/heavy_keys.py r6_key9152 > $O/hk_dbg.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > $O/lin_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_r0.log 2>&1 || exit 1
for RK in 3 4 6; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --seed-rank $RK > $O/bench_r$RK.log 2>&1 || exit 1
done
