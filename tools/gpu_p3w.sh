# phase-3 concurrency sweep on the full C5 history
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in 128 256 512 1024; do
  JH_P3_WAVES=$w JH_DEBUG=1 timeout -k 10 200 python -u tools/exp_c5_budget.py 1000 1048576 > gpurun_out/p3w_full_$w.log 2>&1 || exit 1
done
