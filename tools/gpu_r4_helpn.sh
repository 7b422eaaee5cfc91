# Round 4: late-helper count (jh_lin_opts.helpers 32 default / 48 / 64 / 96)
# and no helper delay (flag 16) on C3 ranks 0 / 7 / 3.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_helpn.sh <outdir>
O=${1:-gpurun_out/r4helpn}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1"
for rk in 0 7 3; do
  timeout -k 10 120 $B --seed-rank $rk > $O/c3r${rk}_h32.json 2> $O/c3r${rk}_h32.err || exit 1
  for h in 48 64 96; do
    timeout -k 10 120 $B --seed-rank $rk --opt helpers=$h > $O/c3r${rk}_h$h.json 2> $O/c3r${rk}_h$h.err || exit 1
  done
  timeout -k 10 120 $B --seed-rank $rk --opt flags=16 > $O/c3r${rk}_now.json 2> $O/c3r${rk}_now.err || exit 1
done
exit 0
