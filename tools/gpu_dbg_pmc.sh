# cycle accounting of the bench (JH_DEBUG=2), then SQ counters of the phase-1 search
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
JH_DEBUG=2 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-parity > gpurun_out/bench_dbg.log 2>&1 && \
bash tools/gpu_pmc.sh
