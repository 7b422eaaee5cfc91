# Round 4: the counter pack with each row's slot and kind kept in registers
# (HEAD) against the committed pack (variants/libjh_cnthead.so), alternating;
# the counter / set parity tests.
#   gpurun --timeout 900 -- bash tools/gpu_r4_cnt.sh <outdir>
O=${1:-gpurun_out/r4cnt}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py > $O/counter_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in new old new2 old2; do :; done
for v in r2 r1 r2b r1b; do
  L=$V/libjh_cntreg2.so; case $v in r1*) L=$V/libjh_cntreg.so;; esac
  JH_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2_$v -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --no-cpu > $R/$O/c2_$v.log 2>&1 || exit 1
done
exit 0
