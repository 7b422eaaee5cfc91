# Phase-1 / phase-2 timeline of the C3 check (JH_DEFER_TIMES=1): when the
# heaviest deferred keys are handed on, when the sequential search takes them.
#   gpurun -- bash tools/gpu_timeline.sh <outdir> [seed-rank ...]
O=${1:-gpurun_out/timeline}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for RK in ${@:-0}; do
  JH_DEFER_TIMES=1 JH_DEBUG=1 timeout -k 10 120 python -u tools/run_once.py c3 3 $RK > $O/rank$RK.log 2>&1 || exit 1
done
