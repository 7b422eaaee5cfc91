# Round-end evidence at HEAD: every GPU test, smoke, the bench line (C3 with CPU baseline + parity),
# rocprofv3 kernel stats of the bench, C4 shard and C5 lines (parity), rank 4/6 rehearsals.
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fin/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/fin/bench_c3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fin/kt -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 > $R/gpurun_out/fin/kt.log 2>&1 || exit 1
cd $R
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --steps 3 --warmup 1 --seed-rank 6 > gpurun_out/fin/bench_r6.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --steps 3 --warmup 1 --seed-rank 4 > gpurun_out/fin/bench_r4.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 500 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/fin/bench_c4.log 2>&1 || exit 1
JH_DEBUG=1 timeout -k 10 500 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/fin/bench_c5.log 2>&1
