O=gpurun_out/help2
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
JH_DEBUG=4 timeout -k 10 120 python -u tools/run_once.py c3 2 0 > $O/r0.log 2>&1 || exit 1
JH_DEBUG=4 timeout -k 10 120 python -u tools/run_once.py c3 2 3 > $O/r3.log 2>&1 || exit 1
JH_DEBUG=4 timeout -k 10 120 python -u tools/run_once.py c3 2 6 > $O/r6.log 2>&1
