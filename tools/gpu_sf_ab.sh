cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/sfab
timeout -k 10 300 python -u -m pytest tests/test_gpu_set_full.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sfab/tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sfab/kt -o sf -- python3 $R/tools/bench_set_full.py --steps 3 --no-cpu > $R/gpurun_out/sfab/kt.log 2>&1
