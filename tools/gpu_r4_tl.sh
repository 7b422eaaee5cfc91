# Round 4: default-schedule C3 timeline (JH_DEFER_TIMES: [jh-last] = the
# keys that end last), the C3 rank-0 bench, then the GPU test suite.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_tl.sh <outdir>
O=${1:-gpurun_out/r4tl}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
timeout -k 10 120 $B > $O/c3.json 2> $O/c3.err || exit 1
JH_LIB=$V/libjh_tune.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl.json 2> $O/tl.err || exit 1
JH_LIB=$V/libjh_tune.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank 3 > $O/tl_r3.json 2> $O/tl_r3.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
exit 0
