# A/B: CAS vs plain-store HBM memo inserts on the full C5 history (phase timings)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
JH_DEBUG=1 timeout -k 10 200 python -u tools/exp_c5_budget.py 1000 1048576 > gpurun_out/ab_cas.log 2>&1 || exit 1
JH_LIB=jepsen_amd/variants/libjh_plain.so JH_DEBUG=1 timeout -k 10 200 python -u tools/exp_c5_budget.py 1000 1048576 > gpurun_out/ab_plain.log 2>&1
