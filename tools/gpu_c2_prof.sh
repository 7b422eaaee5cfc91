# C2 streaming kernels: bench line + rocprofv3 kernel stats, and the C4 bench
# line (one global history sharded by the cost model), one gpurun call.
#   gpurun -- bash tools/gpu_c2_prof.sh <outdir>
O=${1:-gpurun_out/c2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 300 python -u tools/bench_c2.py --no-cpu > $O/bench_c2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/tools/bench_c2.py --no-cpu --steps 3 > $R/$O/kt.log 2>&1 || exit 1
cd $R
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > $O/bench_c4.log 2>&1
