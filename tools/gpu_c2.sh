# C2: counter + set on 100M-entry histories: bench lines and a rocprofv3 kernel summary
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/c2
timeout -k 10 500 python -u tools/bench_c2.py > gpurun_out/c2/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c2/kt -o c2 -- python3 $R/tools/bench_c2.py --steps 3 --no-cpu > $R/gpurun_out/c2/kt.log 2>&1
