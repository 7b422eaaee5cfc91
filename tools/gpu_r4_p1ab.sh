# Round 4: phase-1 memo variants (legacy hash table vs per-key blocks, with
# and without a 5-waves-per-SIMD register cap) on C3 rank 0 with the round-3
# schedule, then the streaming pass's per-key timeline (JH_DEFER_TIMES) with
# and without the early LEAN grid / helpers, then the block memo's DFS stats
# and the FETCH_SIZE / WRITE_SIZE passes of k_lin_dfs<true>.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_p1ab.sh <outdir>
O=${1:-gpurun_out/r4p1ab}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
for v in p1legacy p1blk p1blk5; do
  JH_LIB=$V/libjh_$v.so timeout -k 10 120 $B --opt flags=256 > $O/c3_$v.json 2> $O/c3_$v.err || exit 1
done
JH_LIB=$V/libjh_p1legacy.so timeout -k 10 120 $B > $O/c3_p1legacy_stream.json 2> $O/c3_p1legacy_stream.err || exit 1
JH_LIB=$V/libjh_p1legacy.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_stream.json 2> $O/tl_stream.err || exit 1
JH_LIB=$V/libjh_p1legacy.so JH_DEFER_TIMES=1 JH_EARLY_LEAN=0 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_stream_e0.json 2> $O/tl_stream_e0.err || exit 1
JH_LIB=$V/libjh_p1legacy.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity --opt flags=256 > $O/tl_legacy.json 2> $O/tl_legacy.err || exit 1
JH_LIB=$V/libjh_dfsstats.so JH_DEBUG=2 timeout -k 10 200 python -u tools/run_once.py c3 1 0 > $O/dfsstats_c3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/$O/pmc && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lin_dfs<true>" -d $R/$O/pmc/fetch -o fetch --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/pmc/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_lin_dfs<true>" -d $R/$O/pmc/write -o write --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/pmc/write.log 2>&1 || exit 1
exit 0
