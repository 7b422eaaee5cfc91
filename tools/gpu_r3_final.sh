# Round-3 evidence at HEAD: the whole -m gpu suite, smoke, the bench lines
# (C3 with both CPU baselines, C3 ranks 3 / 6, C4 shard, C5, C2 with CPU
# baselines), rocprofv3 kernel stats of C3 / C5, and FETCH_SIZE / WRITE_SIZE
# passes of the C3 phase-1 and phase-2 kernels (traffic files) and a TCC pass
# over C5's search kernels.
#   gpurun --timeout 1200 -- bash tools/gpu_r3_final.sh <outdir>
O=${1:-gpurun_out/r3final}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --seed-rank 3 > $O/bench_c3_rank3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --seed-rank 6 > $O/bench_c3_rank6.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > $O/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $O/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_c2.py > $O/bench_c2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/$O/ks_c3 -o c3 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity > $R/$O/ks_c3.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/$O/ks_c5 -o c5 --output-format csv -- python3 $R/bench.py --workload c5 --steps 1 --warmup 0 --no-cpu --e2e 0 --no-parity > $R/$O/ks_c5.log 2>&1 || exit 1
for k in "k_lin_seq_lw" "k_lin_dfs<"; do
  n=$(echo "$k" | tr -c 'a-z0-9_\n' '_')
  mkdir -p $R/$O/pmc_c3_$n && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$k" -d $R/$O/pmc_c3_$n/fetch -o fetch --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/pmc_c3_$n/fetch.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$k" -d $R/$O/pmc_c3_$n/write -o write --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/pmc_c3_$n/write.log 2>&1 || exit 1
done
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_lin_seq_lw|k_lin_xw" -d $R/$O/pmc_c5_tcc -o tcc --output-format csv -- python3 $R/tools/run_once.py c5 1 0 > $R/$O/pmc_c5_tcc.log 2>&1 || exit 1
exit 0
