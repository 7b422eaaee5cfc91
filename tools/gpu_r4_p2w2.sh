# Round 4: phase 2 at one wave per CU (p2_waves_per_cu = 1) on C3 ranks 4 / 6 / 0, alternating.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_p2w2.sh <outdir>
O=${1:-gpurun_out/r4p2w2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1"
for rep in 1 2; do
for rk in 4 6 0; do
  timeout -k 10 120 $B --seed-rank $rk > $O/c3r${rk}_w4_$rep.json 2> $O/c3r${rk}_w4_$rep.err || exit 1
  timeout -k 10 120 $B --seed-rank $rk --opt p2_waves_per_cu=1 > $O/c3r${rk}_w1_$rep.json 2> $O/c3r${rk}_w1_$rep.err || exit 1
done
done
exit 0
