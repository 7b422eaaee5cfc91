# Round 4 final evidence at HEAD. Part a: the GPU suite, smoke(), the
# default bench line (CPU baselines, parity) and its kernel stats. Part b:
# C3 ranks 1-7, C4, C5 and C2 lines, C2 kernel stats. Part c2: the C2 lines
# and kernel stats only.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_final.sh <outdir> a|b|c2
O=${1:-gpurun_out/r4final}; PART=${2:-a}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
if [ $PART = a ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c3prof -o c3 -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity > $R/$O/c3prof.log 2>&1 || exit 1
exit 0
fi
if [ $PART = c2 ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2prof -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 > $R/$O/bench_c2.log 2>&1 || exit 1
exit 0
fi
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
for rk in 1 2 3 4 5 6 7; do
  timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}.json 2> $O/c3r${rk}.err || exit 1
done
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2prof -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 > $R/$O/bench_c2.log 2>&1 || exit 1
exit 0
