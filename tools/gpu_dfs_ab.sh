# search-kernel change: the lin / limits parity tests, then C3 ranks 0 / 3 / 6
# and C5 of the in-tree build and of jepsen_amd/variants/libjh_<v>.so
#   gpurun --timeout 1200 -- bash tools/gpu_dfs_ab.sh <outdir> [variants...]
O=${1:-gpurun_out/dfsab}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_lin.py tests/test_gpu_limits.py > $O/lin_tests.log 2>&1 || exit 1
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
for rk in 0 3 6; do
  timeout -k 10 200 $B --seed-rank $rk > $O/new_r$rk.log 2>&1 || exit 1
  for v in "$@"; do
    JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 200 $B --seed-rank $rk > $O/${v}_r$rk.log 2>&1 || exit 1
  done
done
C="python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --e2e 0 --no-parity"
timeout -k 10 150 $C > $O/c5_new.log 2>&1 || exit 1
for v in "$@"; do
  JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 150 $C > $O/c5_$v.log 2>&1 || exit 1
done
exit 0
