# Round 4: C5 at insert budget 2^24 (one step, no warm-up).
#   gpurun --timeout 1200 -- bash tools/gpu_r4_c5b24.sh <outdir>
O=${1:-gpurun_out/r4c5b24}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 1000 python -u bench.py --workload c5 --steps 1 --warmup 0 --budget 16777216 --no-cpu --e2e 0 --no-parity > $O/c5_b24.json 2> $O/c5_b24.err || exit 1
exit 0
