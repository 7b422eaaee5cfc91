# Round 3: after a search-kernel change -- the BFS / lin parity tests first,
# then the C3 rank 0 / 3 / 6 lines and a per-workgroup BFS accounting run
# (tuning build, JH_DEBUG=2) of rank 3; optionally the C2 script after it.
#   gpurun --timeout 1200 -- bash tools/gpu_r3_lin.sh <outdir> [c2]
O=${1:-gpurun_out/r3lin}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_lin.py -k "bfs_exact or linear or frontier or heavy_key or c3_scale" > $O/bfs_tests.log 2>&1 || exit 1
timeout -k 10 700 $T tests/test_gpu_lin.py tests/test_gpu_limits.py tests/test_gpu_configs.py > $O/lin_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --seed-rank 3 > $O/bench_c3_rank3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --seed-rank 6 > $O/bench_c3_rank6.log 2>&1 || exit 1
JH_LIB=$R/jepsen_amd/variants/libjh_tune.so JH_DEBUG=2 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank 3 > $O/dbg_rank3.log 2>&1 || exit 1
if [ "$2" = "c2" ]; then bash tools/gpu_c2.sh $O/c2 || exit 1; fi
exit 0
