# C2 streaming kernels: their GPU tests, the bench lines and rocprofv3 kernel
# stats, one gpurun call.   gpurun -- bash tools/gpu_c2_prof.sh <outdir>
O=${1:-gpurun_out/c2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "counter or set or c2" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_c2.py --no-cpu > $O/bench_c2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/tools/bench_c2.py --no-cpu --steps 3 > $R/$O/kt.log 2>&1
