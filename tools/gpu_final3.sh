# Round-end evidence at HEAD: every GPU test, smoke, the bench line (C3, CPU baseline + parity),
# rocprofv3 kernel stats of the bench, set-full and queue bench lines.
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/fin3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fin3/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin3/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/fin3/bench_c3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fin3/kt -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 > $R/gpurun_out/fin3/kt.log 2>&1 || exit 1
cd $R
timeout -k 10 300 python -u tools/bench_set_full.py > gpurun_out/fin3/bench_set_full.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_queue.py > gpurun_out/fin3/bench_queue.log 2>&1
