# The workgroup engine racing the BFS (JH_WG=2) against the default race:
# heavy keys one by one, the C3 bench line, and the lin parity tests on JH_WG=2.
O=${1:-gpurun_out/wgr}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for W in 0 2; do
  JH_WG=$W timeout -k 10 200 python -u tools/heavy_keys.py > $O/hk_$W.log 2>&1 || exit 1
  JH_WG=$W timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_$W.log 2>&1 || exit 1
done
JH_WG=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -q --timeout 300 --timeout-method thread > $O/lin_tests.log 2>&1
