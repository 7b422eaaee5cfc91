# Round 4: four / two 16-byte loads in flight per thread in the range scans
# (k_cnt_prange, k_set_range) and two row pairs per step in k_set_scan, against
# the committed kernels (head), alternating; counter / set parity.
#   gpurun --timeout 900 -- bash tools/gpu_r4_unroll.sh <outdir>
O=${1:-gpurun_out/r4unroll}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
for v in u4 u4s2 u2 u1; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py > $O/tests_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in head u1 u2 u4 u4s2; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
exit 0
