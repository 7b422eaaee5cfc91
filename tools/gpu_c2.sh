# C2 after a change: counter / set parity tests, the C2 bench lines (with the
# CPU baseline) and the kernel stats of one bench run.
#   gpurun --timeout 900 -- bash tools/gpu_c2.sh <outdir>
O=${1:-gpurun_out/c2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_counter_set.py -x -v --timeout 200 --timeout-method thread > $O/cs_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_c2.py > $O/bench_c2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/$O/ks -o c2 --output-format csv -- python3 $R/tools/bench_c2.py --steps 3 --warmup 1 --no-cpu > $R/$O/ks.log 2>&1 || exit 1
exit 0
