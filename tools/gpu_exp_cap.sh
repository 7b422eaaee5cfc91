# C5 memo footprint experiment: same work, 1x / 2x / 4x HBM memo capacity per search
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 0 1 2; do
  JH_MEMO_CAP_SHIFT=$c JH_DEBUG=1 timeout -k 10 200 python -u tools/exp_c5_budget.py 1000 1048576 > gpurun_out/exp_cap_$c.log 2>&1 || exit 1
done
rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1 || true
