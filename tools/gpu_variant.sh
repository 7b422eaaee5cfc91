# A/B of a jh_lin.hip variant built by tools/build_variants.sh: lin parity tests
# on the variant, then rank 0/3/6 timings of the variant and of the default lib.
#   gpurun -- bash tools/gpu_variant.sh <outdir> <variant-name>
O=${1:-gpurun_out/var}; V=${2:-t1024}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
JH_LIB=$R/jepsen_amd/variants/libjh_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > $O/lin_tests_$V.log 2>&1 || exit 1
for RK in 0 3 6; do
  JH_LIB=$R/jepsen_amd/variants/libjh_$V.so timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --seed-rank $RK > $O/bench_${V}_r$RK.log 2>&1 || exit 1
done
