# Round 4: the set byte-map pass from the scan's per-row codes (JH_SET_CODE=1:
# 2 + 16 bytes per row pair instead of 48) against the three-column pass (sc0),
# alternating, both software-pipelined; then (scw0 / scw1) one 16-byte store of eight lanes' codes (JH_SET_CODE_WIDE); parity.
#   gpurun --timeout 900 -- bash tools/gpu_r4_scode.sh <outdir>
O=${1:-gpurun_out/r4scode}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
for v in scw1; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py > $O/tests_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in scw0 scw1; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
exit 0
