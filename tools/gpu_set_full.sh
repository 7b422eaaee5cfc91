# set-full: GPU parity tests, bench line, rocprofv3 kernel stats
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/sf
timeout -k 10 400 python -u -m pytest tests/test_gpu_set_full.py -x -v --timeout 200 --timeout-method thread > gpurun_out/sf/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_set_full.py > gpurun_out/sf/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sf/kt -o sf -- python3 $R/tools/bench_set_full.py --steps 3 --no-cpu > $R/gpurun_out/sf/kt.log 2>&1
