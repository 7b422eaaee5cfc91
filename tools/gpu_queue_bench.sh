# queue bench lines + rocprofv3 kernel stats
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/qb
timeout -k 10 400 python -u tools/bench_queue.py > gpurun_out/qb/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/qb/kt -o q -- python3 $R/tools/bench_queue.py --steps 3 --no-cpu --enqueues 1000000 > $R/gpurun_out/qb/kt.log 2>&1
