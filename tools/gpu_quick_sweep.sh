# phase-1 quick budget at HEAD: C3 ranks 0 / 3 / 6 and the C4 shard at the
# default (8 192) and the given values (jh_lin_opts.quick_budget via --opt)
#   gpurun -- bash tools/gpu_quick_sweep.sh <outdir> 7168 10240
O=${1:-gpurun_out/quick}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
for qb in 0 "$@"; do
  o=""; [ "$qb" != 0 ] && o="--opt quick_budget=$qb"
  for rk in 0 3 6; do
    timeout -k 10 200 $B --seed-rank $rk $o > $O/q${qb}_r$rk.log 2>&1 || exit 1
  done
  timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity $o > $O/q${qb}_c4.log 2>&1 || exit 1
done
exit 0
