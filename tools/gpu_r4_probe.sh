# Round-4 first probe: the counter parity tests (ADVICE r3 fix), phase-1
# FETCH_SIZE / WRITE_SIZE of k_lin_dfs<true> on C3 at HEAD, and a
# -DJH_DFS_STATS tuning build's per-phase counts (evictions, entries moved to
# the HBM table, stack spills / refills, HBM probes) on the same history.
#   gpurun --timeout 900 -- bash tools/gpu_r4_probe.sh <outdir>
O=${1:-gpurun_out/r4probe}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_counter_set.py -x -v --timeout 120 --timeout-method thread > $O/counter_tests.log 2>&1 || exit 1
JH_LIB=$R/jepsen_amd/variants/libjh_dfsstats.so JH_DEBUG=2 timeout -k 10 200 python -u tools/run_once.py c3 1 0 > $O/dfsstats_c3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
k="k_lin_dfs<true>"
mkdir -p $R/$O/pmc_c3_dfs && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lin_dfs<true>" -d $R/$O/pmc_c3_dfs/fetch -o fetch --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/pmc_c3_dfs/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_lin_dfs<true>" -d $R/$O/pmc_c3_dfs/write -o write --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/pmc_c3_dfs/write.log 2>&1 || exit 1
exit 0
