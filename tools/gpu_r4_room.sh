# Round 4: the BFS set's per-insert retry of a refused batch reservation
# (HEAD) against none (JH_BFS_ROOM_EXACT=0): C4, C3 ranks 0/3/6; quick
# budget re-check on rank 0; the N = 2 pool rehearsal.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_room.sh <outdir>
O=${1:-gpurun_out/r4room}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
for rep in 1 2; do
  timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_head_$rep.json 2> $O/c4_head_$rep.err || exit 1
  JH_LIB=$V/libjh_room0.so timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_room0_$rep.json 2> $O/c4_room0_$rep.err || exit 1
done
for rk in 0 3 6; do
  timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_head.json 2> $O/c3r${rk}_head.err || exit 1
  JH_LIB=$V/libjh_room0.so timeout -k 10 120 $B --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}_room0.json 2> $O/c3r${rk}_room0.err || exit 1
done
for qb in 7168 10240; do
  timeout -k 10 120 $B --steps 5 --warmup 1 --opt quick_budget=$qb > $O/c3r0_q$qb.json 2> $O/c3r0_q$qb.err || exit 1
done
JH_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/rehearse_n2_pool.log 2>&1 || exit 1
exit 0
