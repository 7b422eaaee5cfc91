# One JH_DEBUG=2 run of a C3 rank history (BFS per-workgroup accounting).
#   gpurun -- bash tools/gpu_bfs_dbg1.sh <outdir> <seed-rank>
O=${1:-gpurun_out/bfsdbg1}; RK=${2:-3}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
JH_DEBUG=2 timeout -k 10 120 python -u tools/run_once.py c3 1 $RK > $O/dbg_r$RK.log 2>&1
