# Round 4: phase 1's instruction mix and issue (one SQ --pmc pass over
# k_lin_dfs<true, false> on C3 rank 0).
#   gpurun --timeout 600 -- bash tools/gpu_r4_p1sq.sh <outdir>
O=${1:-gpurun_out/r4p1sq}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --kernel-include-regex "k_lin_dfs<true, false>" -d $R/$O/sq -o sq --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/sq.log 2>&1 || exit 1
exit 0
