# Round 4: phase 2 at one sequential wave per CU with the 128 KB memo
# (jh_lin_opts.p2_waves_per_cu = 1) against four per CU (default), C3 ranks 0 / 7 / 3, C4.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_p2w.sh <outdir>
O=${1:-gpurun_out/r4p2w}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1"
for rep in 1 2; do
for rk in 0 7 3; do
  timeout -k 10 120 $B --seed-rank $rk > $O/c3r${rk}_w4_$rep.json 2> $O/c3r${rk}_w4_$rep.err || exit 1
  timeout -k 10 120 $B --seed-rank $rk --opt p2_waves_per_cu=1 > $O/c3r${rk}_w1_$rep.json 2> $O/c3r${rk}_w1_$rep.err || exit 1
done
done
timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --no-parity --workload c4 --steps 3 --warmup 1 --opt p2_waves_per_cu=1 > $O/c4_w1.json 2> $O/c4_w1.err || exit 1
exit 0
