# HIP runtime + kernel trace stats of the queue bench (where the wall time outside kernels goes)
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/qt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/qt/t -o q -- python3 $R/tools/bench_queue.py --steps 3 --no-cpu --enqueues 1000000 > $R/gpurun_out/qt/t.log 2>&1
