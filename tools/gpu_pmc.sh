# HBM traffic of one kernel on one bench workload history: separate
# FETCH_SIZE and WRITE_SIZE rocprofv3 passes (one counter per pass,
# MI355X_MICROARCH.md), each over `tools/run_once.py <workload> 1 <rank>`
# (which prints its own summary). Run tools/pmc_traffic.py on the CPU side
# after the call.
#   gpurun -- bash tools/gpu_pmc.sh <workload> <kernel-regex> <outdir> [rank]
W=${1:-c3}; K=${2:-k_lin_seq3<}; O=${3:-gpurun_out/pmc_$W}; RK=${4:-0}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $R/$O/fetch -o fetch --output-format csv -- python3 $R/tools/run_once.py $W 1 $RK > $R/$O/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $R/$O/write -o write --output-format csv -- python3 $R/tools/run_once.py $W 1 $RK > $R/$O/write.log 2>&1
