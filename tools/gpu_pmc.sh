# rocprofv3 PMC counters of the phase-1 search kernel, one counter group per pass
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM --kernel-include-regex "k_lin_dfs" -d $R/gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 $R/tools/run_c3_once.py > $R/gpurun_out/pmc/p1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA --kernel-include-regex "k_lin_dfs" -d $R/gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 $R/tools/run_c3_once.py > $R/gpurun_out/pmc/p2.log 2>&1
