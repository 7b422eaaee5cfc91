# Round 4: the counter spill pass on per-chunk first-row tables (JH_SPILL_TAB=1)
# against the eight-row walk (tab0), alternating; counter / set parity for
# both (incl. test_counter_walk_across_chunks).
#   gpurun --timeout 900 -- bash tools/gpu_r4_tab.sh <outdir>
O=${1:-gpurun_out/r4tab}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
for v in tab1 tab0; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py > $O/tests_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in tab0 tab1; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
exit 0
