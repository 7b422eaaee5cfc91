# Round 4: the counter's spill pass with the process offset and f2 carried in
# the spill entry, lanes per chunk 16 / 32 / 64 (and 16 rows per walk step),
# against the eight-row walk of the old entry (sv8), alternating; parity.
#   gpurun --timeout 900 -- bash tools/gpu_r4_sl.sh <outdir>
O=${1:-gpurun_out/r4sl}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
for v in sl16 sl32 sl64; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py -k counter > $O/tests_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in sv8 sl16 sl32 sl64 sl32v16; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
exit 0
