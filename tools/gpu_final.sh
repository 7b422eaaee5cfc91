# Round-end evidence: smoke, the bench line (C3 with CPU baseline + parity), rocprofv3 kernel
# stats of the bench, FETCH_SIZE / WRITE_SIZE passes of the phase-1 search, C2 lines + stats,
# C4 / C5 lines. (GPU tests run separately: tools/gpu_tests.sh.)
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench_c3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/kt -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 > $R/gpurun_out/final/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lin_dfs" -d $R/gpurun_out/final/fetch -o fetch --output-format csv -- python3 $R/tools/run_c3_once.py 10000 2 > $R/gpurun_out/final/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_lin_dfs" -d $R/gpurun_out/final/write -o write --output-format csv -- python3 $R/tools/run_c3_once.py 10000 2 > $R/gpurun_out/final/write.log 2>&1 || exit 1
cd $R
timeout -k 10 500 python -u tools/bench_c2.py > gpurun_out/final/bench_c2.log 2>&1 || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/c2kt -o c2 -- python3 $R/tools/bench_c2.py --steps 3 --no-cpu > $R/gpurun_out/final/c2kt.log 2>&1 || exit 1
cd $R
JH_DEBUG=1 timeout -k 10 400 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/final/bench_c5.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 500 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/final/bench_c4.log 2>&1
