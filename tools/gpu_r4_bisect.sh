# Round 4: C4 across the round-2 -> round-3 commits (git worktrees bis_<c>/)
# to find the phase-2 regression, plus HEAD's C3 / C4 and the lin tests.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_bisect.sh <outdir> <commit>...
O=$1; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for c in "$@"; do
  (cd $R/bis_$c && timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity > $R/$O/c4_$c.json 2> $R/$O/c4_$c.err) || exit 1
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/c4_head.json 2> $O/c4_head.err || exit 1
timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/c3_head.json 2> $O/c3_head.err || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lin.py > $O/lin_tests.log 2>&1 || exit 1
exit 0
