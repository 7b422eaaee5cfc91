# k_lin_xw instruction mix on C5 (one rocprofv3 --pmc pass, SQ counters only):
# instructions and wave cycles per insert, against the JH_XW_PROF split
#   gpurun -- bash tools/gpu_xw_pmc.sh <outdir>
O=${1:-gpurun_out/xwpmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_lin_xw" -d $R/$O/sq -o sq --output-format csv -- python3 $R/tools/run_once.py c5 1 0 > $R/$O/sq.log 2>&1
