# k_lin_bfs change: the BFS parity tests, then C3 ranks 0 / 3 / 6 of the
# in-tree build and of jepsen_amd/variants/libjh_<v>.so for each v given
#   gpurun --timeout 900 -- bash tools/gpu_bfs_ab.sh <outdir> [variants...]
O=${1:-gpurun_out/bfsab}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_lin.py -k "bfs_exact or linear or frontier or heavy_key or c3_scale" > $O/bfs_tests.log 2>&1 || exit 1
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
for rk in 0 3 6; do
  timeout -k 10 200 $B --seed-rank $rk > $O/new_r$rk.log 2>&1 || exit 1
  for v in "$@"; do
    JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 200 $B --seed-rank $rk > $O/${v}_r$rk.log 2>&1 || exit 1
  done
done
exit 0
