# Round 4: the counter tile scan with 1 / 2 / 4 tiles per block (one barrier for
# all, every tile's words loaded first) and 2 tiles capped at 80 VGPRs, against
# the one-tile scan of e2de750 (sl32), alternating; parity.
#   gpurun --timeout 900 -- bash tools/gpu_r4_ts.sh <outdir>
O=${1:-gpurun_out/r4ts}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
for v in ts2 ts4 ts2w6; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py -k counter > $O/tests_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in sl32 ts1 ts2 ts4 ts2w6; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
exit 0
