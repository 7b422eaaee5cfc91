# Round 4: grid caps of k_set_scan / k_set_bytes_code (4096 / 16384 default,
# 8192 / 8192, 2048 / 32768, 16384 / 4096), alternating; set parity for one.
#   gpurun --timeout 900 -- bash tools/gpu_r4_sgrid.sh <outdir>
O=${1:-gpurun_out/r4sgrid}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
JH_LIB=$V/libjh_g3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py -k set > $O/tests_g3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in g0 g1 g2 g3; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
exit 0
