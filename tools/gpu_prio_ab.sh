# A/B of phase-1 issue priorities (JH_P1_PRIO, tuning build): C3 rank 0 / 3
# lines per threshold; then the counter's per-phase profile and the C2 script.
#   gpurun --timeout 1500 -- bash tools/gpu_prio_ab.sh <outdir>
O=${1:-gpurun_out/prio}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for p in 0 256 1024 2048; do
  for rk in 0 3; do
    JH_LIB=$R/jepsen_amd/variants/libjh_tune.so JH_P1_PRIO=$p timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank $rk > $O/c3_p${p}_r${rk}.log 2>&1 || exit 1
  done
done
JH_LIB=$R/jepsen_amd/variants/libjh_cntprof.so timeout -k 10 300 python -u tools/bench_c2.py --steps 3 --warmup 1 --no-cpu > $O/cprof.log 2>&1 || exit 1
bash tools/gpu_c2.sh $O/c2 || exit 1
exit 0
