# PMC of the phase-3 search on C5-shaped keys at two concurrencies (one counter group per pass)
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for w in 64 1024; do
  o=$R/gpurun_out/pmc_c5/w$w; mkdir -p $o
  JH_P3_WAVES=$w timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU --kernel-include-regex "k_lin_seq3" -d $o/p1 -o p1 --output-format csv -- python3 $R/tools/exp_c5_budget.py 300 1048576 > $o/p1.log 2>&1 || exit 1
  JH_P3_WAVES=$w timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_lin_seq3" -d $o/p2 -o p2 --output-format csv -- python3 $R/tools/exp_c5_budget.py 300 1048576 > $o/p2.log 2>&1 || exit 1
done
