# Round 4: phase 1 at 7 waves per SIMD (VGPR cap 72) with the 2 KB / 1 KB
# Bloom filter, against HEAD (6 waves, 2 KB): C3 ranks 0 / 7, C4; lin tests
# on the best-looking variant are run separately.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_w7.sh <outdir>
O=${1:-gpurun_out/r4w7}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --no-cpu --e2e 0 --no-parity"
for rep in 1 2; do
  for v in head w7 w7b13 w6b13; do
    L=""; [ $v != head ] && L=$V/libjh_$v.so
    JH_LIB=$L timeout -k 10 120 $B --steps 5 --warmup 1 > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 1
  done
done
for v in head w7 w7b13; do
  L=""; [ $v != head ] && L=$V/libjh_$v.so
  JH_LIB=$L timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $O/c4_$v.json 2> $O/c4_$v.err || exit 1
done
exit 0
