# Round 4 measurements at HEAD: C4 shard, C5 at insert budgets 2^20 / 2^22,
# the N = 2 rehearsal of the two-stage pool (every rank on cuda:0 over gloo),
# and the FETCH_SIZE / WRITE_SIZE passes of phase 1 and phase 2 on C3 seed 3.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_meas.sh <outdir> a|b
O=${1:-gpurun_out/r4meas}
PART=${2:-a}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
if [ $PART = a ]; then
# counter pack: the pipelined kernel (2 blocks / CU, default; 1 block: cw0; 3 blocks: cw6) against round 3's
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py > $O/counter_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in head cw0 cw6 r3; do
  L=""; T=$R; [ $v = cw0 ] && L=$V/libjh_cw0.so; [ $v = cw6 ] && L=$V/libjh_cw6.so; [ $v = r3 ] && T=$R/r3ref
  JH_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_$v -o c2 -- python3 $T/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_$v.log 2>&1 || exit 1
done
cd $R
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 --budget 1048576 > $O/c4_b20.json 2> $O/c4_b20.err || exit 1
timeout -k 10 200 $B --workload c5 --steps 1 --warmup 1 > $O/c5_b20.json 2> $O/c5_b20.err || exit 1
JH_LIB=$V/libjh_xw4.so timeout -k 10 200 $B --workload c5 --steps 1 --warmup 1 > $O/c5_b20_xw4.json 2> $O/c5_b20_xw4.err || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_lin.py tests/test_c_harness.py -k "c5 or xw or wide or frontier" > $O/xw_tests.log 2>&1 || exit 1
timeout -k 10 300 $B --workload c5 --steps 1 --warmup 0 --budget 4194304 > $O/c5_b22.json 2> $O/c5_b22.err || exit 1
exit 0
fi
C="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
# C4 on this box: rounds 2 and 3 (git worktrees r2ref/, r3ref/) against HEAD
for t in r2ref r3ref; do
  (cd $R/$t && timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity > $R/$O/c4_$t.json 2> $R/$O/c4_$t.err) || exit 1
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/c4_head.json 2> $O/c4_head.err || exit 1
for rep in 1 2; do
  timeout -k 10 120 $C > $O/c3_head_$rep.json 2> $O/c3_head_$rep.err || exit 1
  JH_LIB=$V/libjh_p1w6.so timeout -k 10 120 $C > $O/c3_p1w6_$rep.json 2> $O/c3_p1w6_$rep.err || exit 1
done
JH_LIB=$V/libjh_p1w6.so timeout -k 10 120 $C --seed-rank 3 > $O/c3r3_p1w6.json 2> $O/c3r3_p1w6.err || exit 1
for rk in 1 2 3 4 5 6 7; do
  timeout -k 10 120 $C --seed-rank $rk > $O/c3r${rk}_head.json 2> $O/c3r${rk}_head.err || exit 1
done
JH_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/rehearse_n2_pool.log 2>&1 || exit 1
JH_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity --pool 0 > $O/rehearse_n2_nopool.log 2>&1 || exit 1
bash tools/gpu_pmc.sh c3 "k_lin_dfs<true, false>" $O/pmc_p1 0 || exit 1
bash tools/gpu_pmc.sh c3 "k_lin_seq_lw<false>" $O/pmc_p2 0 || exit 1
exit 0
