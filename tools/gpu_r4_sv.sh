# Round 4: the counter's spill walk, rows per step (JH_SPILL_VEC 0 / 4 / 8 / 16),
# alternating; counter parity for the vector walks.
#   gpurun --timeout 900 -- bash tools/gpu_r4_sv.sh <outdir>
O=${1:-gpurun_out/r4sv}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
for v in sv8 sv16; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py -k counter > $O/tests_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in sv0 sv4 sv8 sv16; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
exit 0
