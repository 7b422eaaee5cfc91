# round 5, late: the whole GPU suite + smoke + the C3 line at HEAD (packed
# host-buffer staging), then the phase-1 duplicate-write A/B
O=gpurun_out/r5p
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 200 python -u tools/bench_c2.py --steps 5 --warmup 1 --e2e > $O/bench_c2.log 2>&1 || exit 1
bash tools/gpu_dup.sh
