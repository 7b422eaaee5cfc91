# k_lin_xw change: the wide-window parity tests (of the build named by $1's
# variant, default the in-tree one), then C5 lines of the in-tree build, each
# jepsen_amd/variants/libjh_<v>.so named after the outdir, and the previous
# build (variants/libjh_old.so)
#   gpurun --timeout 900 -- bash tools/gpu_xw.sh <outdir> [test-variant] [bench variants...]
O=${1:-gpurun_out/xw}; TV=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
T="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
if [ -n "$TV" ] && [ "$TV" != "-" ]; then export JH_LIB=$R/jepsen_amd/variants/libjh_$TV.so; fi
timeout -k 10 500 $T tests/test_gpu_lin.py tests/test_gpu_configs.py -k "wider_than_64 or c5_shape or c5_full" > $O/xw_tests.log 2>&1 || exit 1
unset JH_LIB
B="python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --e2e 0 --no-parity"
timeout -k 10 150 $B > $O/c5_new.log 2>&1 || exit 1
for v in "$@"; do
  JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 150 $B > $O/c5_$v.log 2>&1 || exit 1
done
exit 0
