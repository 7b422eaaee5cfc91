# Round-2 evidence at HEAD, one gpurun call: every -m gpu test, smoke, the C3
# bench line (parity + both CPU baselines), rocprofv3 kernel stats of the bench,
# phase-2 FETCH/WRITE_SIZE, the C4-shard / C5 / C2 lines, the rank 3 and 6
# rehearsals, and one TCC pass over C5's phase-3 kernel (its plateau).
#   gpurun --timeout 1200 -- bash tools/gpu_round2.sh <outdir>
O=${1:-gpurun_out/round2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --seed-rank 3 > $O/bench_c3_rank3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --seed-rank 6 > $O/bench_c3_rank6.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --e2e 0 > $O/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_c2.py --no-cpu > $O/bench_c2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 > $R/$O/kt.log 2>&1 || exit 1
bash $R/tools/gpu_pmc.sh c3 "k_lin_seq3<" $O/pmc_c3 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-include-regex "k_lin_seq3" -d $R/$O/pmc_c5 -o tcc --output-format csv -- python3 $R/tools/run_once.py c5 1 > $R/$O/pmc_c5_tcc.log 2>&1
exit 0
