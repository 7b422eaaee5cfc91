# rocprofv3 PMC counters of the search kernels (phase 1 + heavy keys), one counter group per pass.
# usage: gpu_pmc.sh [variant ...]   (base = jepsen_amd/libjh.so, else jepsen_amd/variants/libjh_<v>.so)
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "${@:-base}"; do
  lib=$R/jepsen_amd/libjh.so; [ "$v" != base ] && lib=$R/jepsen_amd/variants/libjh_$v.so
  o=$R/gpurun_out/pmc/$v; mkdir -p $o
  JH_LIB=$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM --kernel-include-regex "k_lin_dfs|k_lin_seq" -d $o/p1 -o p1 --output-format csv -- python3 $R/tools/run_c3_once.py > $o/p1.log 2>&1 || exit 1
  JH_LIB=$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA --kernel-include-regex "k_lin_dfs|k_lin_seq" -d $o/p2 -o p2 --output-format csv -- python3 $R/tools/run_c3_once.py > $o/p2.log 2>&1 || exit 1
done
