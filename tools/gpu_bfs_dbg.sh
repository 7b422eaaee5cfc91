# Per-workgroup BFS accounting (JH_DEBUG=2: cycles, rounds, configurations,
# count-pass phases) on the C3 rank histories.
#   gpurun -- bash tools/gpu_bfs_dbg.sh <outdir> [seed-rank ...]
O=${1:-gpurun_out/bfsdbg}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for RK in ${@:-0}; do
  JH_DEBUG=2 timeout -k 10 120 python -u tools/run_once.py c3 1 $RK > $O/rank$RK.log 2>&1 || exit 1
done
