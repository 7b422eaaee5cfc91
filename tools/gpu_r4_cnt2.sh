# Round 4: counter pack A/B -- group masks by per-wave ballots (JH_CNT_BALLOT),
# a 32-bit slot hash (JH_CNT_HASH32), both, the tile scan's prefix load issued
# first (cnt_base vs the committed cnt_head); counter parity per variant; one
# SQ pass over the pack.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_cnt2.sh <outdir>
O=${1:-gpurun_out/r4cnt2}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
for v in cnt_ballot cnt_hash32 cnt_both; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py -k counter > $O/tests_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in cnt_head cnt_base cnt_ballot cnt_hash32 cnt_both; do
    JH_LIB=$V/libjh_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_${v}_$rep -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_${v}_$rep.log 2>&1 || exit 1
  done
done
JH_LIB=$V/libjh_cnt_base.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --kernel-include-regex "k_cnt_pack" -d $R/$O/sq -o sq --output-format csv -- python3 $R/tools/bench_c2.py --steps 2 --warmup 1 --no-cpu > $R/$O/sq.log 2>&1 || exit 1
JH_LIB=$V/libjh_cnt_base.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "k_cnt_pack" -d $R/$O/sq2 -o sq2 --output-format csv -- python3 $R/tools/bench_c2.py --steps 2 --warmup 1 --no-cpu > $R/$O/sq2.log 2>&1 || exit 1
exit 0
