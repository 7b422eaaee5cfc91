# Phase-2 configuration sweep (run_once, last of the calls): quick budget,
# late-helper delay and count, on C3 rank histories and C4/C5.
O=${1:-gpurun_out/p2s}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for cfg in "8192 500 16" "8192 2000 32" "8192 500 32" "8192 1000 16"; do
  set -- $cfg
  echo "rank=0 quick=$1 late=$2 helpers=$3 $(JH_QUICK_BUDGET=$1 JH_HELPER_LATE_US=$2 JH_HELPERS=$3 timeout -k 10 100 python -u tools/run_once.py c3 3 0 2>&1 | tail -1)" >> $O/sweep.log || exit 1
done
for RK in 3 4; do
  echo "rank=$RK quick=8192 $(JH_QUICK_BUDGET=8192 timeout -k 10 100 python -u tools/run_once.py c3 3 $RK 2>&1 | tail -1)" >> $O/sweep.log || exit 1
done
echo "c4 quick=4096 $(timeout -k 10 200 python -u tools/run_once.py c4 2 2>&1 | tail -1)" >> $O/sweep.log || exit 1
echo "c4 quick=8192 $(JH_QUICK_BUDGET=8192 timeout -k 10 200 python -u tools/run_once.py c4 2 2>&1 | tail -1)" >> $O/sweep.log || exit 1
echo "c5 quick=4096 $(timeout -k 10 200 python -u tools/run_once.py c5 1 2>&1 | tail -1)" >> $O/sweep.log || exit 1
echo "c5 quick=8192 $(JH_QUICK_BUDGET=8192 timeout -k 10 200 python -u tools/run_once.py c5 1 2>&1 | tail -1)" >> $O/sweep.log
