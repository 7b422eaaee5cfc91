# Round 4: k_lin_xw on C5 at HEAD (two-slice search): the JH_XW_PROF split
# and one SQ --pmc pass (instruction mix per insert).
#   gpurun --timeout 900 -- bash tools/gpu_r4_xwprof.sh <outdir>
O=${1:-gpurun_out/r4xwprof}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
JH_LIB=$V/libjh_xwprof.so timeout -k 10 200 python -u tools/run_once.py c5 1 0 > $O/xwprof.log 2>&1 || exit 1
bash tools/gpu_xw_pmc.sh $O || exit 1
exit 0
