# Round 4: the gap between phase 1 and the heavy-key pass -- C3 bench
# (p2_start_ms) and a kernel trace of 3 C3 checks (kernel start/end times).
#   gpurun --timeout 900 -- bash tools/gpu_r4_gap.sh <outdir>
O=${1:-gpurun_out/r4gap}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/c3.json 2> $O/c3.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt -o kt -- python3 $R/tools/run_once.py c3 3 0 > $R/$O/kt.log 2>&1 || exit 1
exit 0
