# GPU parity tests, cycle accounting, the full bench line, a rocprofv3
# kernel-trace summary of the bench, and FETCH_SIZE / WRITE_SIZE passes over
# the phase-1 search kernel (one counter per pass, MI355X_MICROARCH.md).
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "not c2_scale" > gpurun_out/gpu_tests.log 2>&1 && \
JH_DEBUG=2 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-parity > gpurun_out/bench_dbg.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kt -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-parity > $R/gpurun_out/prof/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lin_dfs" -d $R/gpurun_out/prof/fetch -o fetch --output-format csv -- python3 $R/tools/run_c3_once.py 10000 2 > $R/gpurun_out/prof/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_lin_dfs" -d $R/gpurun_out/prof/write -o write --output-format csv -- python3 $R/tools/run_c3_once.py 10000 2 > $R/gpurun_out/prof/write.log 2>&1
