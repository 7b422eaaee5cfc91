# Round 4: wide-window :configs tests + the C3 rank-0 A/B of the round-3
# build (git worktree r3ref/, same box) against HEAD with and without the
# streaming pass and with the legacy phase-1 memo, then the streaming
# timeline (JH_DEFER_TIMES, [jh-last] = the last keys to finish).
#   gpurun --timeout 1200 -- bash tools/gpu_r4_ab2.sh <outdir>
O=${1:-gpurun_out/r4ab2}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lin.py -k "frontier_configs or streamed or block_memo" > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
(cd $R/r3ref && timeout -k 10 120 $B > $R/$O/c3_r3ref.json 2> $R/$O/c3_r3ref.err) || exit 1
timeout -k 10 120 $B > $O/c3_head.json 2> $O/c3_head.err || exit 1
timeout -k 10 120 $B --opt flags=256 > $O/c3_head_ns.json 2> $O/c3_head_ns.err || exit 1
JH_LIB=$V/libjh_p1legacy.so timeout -k 10 120 $B --opt flags=256 > $O/c3_p1legacy_ns.json 2> $O/c3_p1legacy_ns.err || exit 1
(cd $R/r3ref && timeout -k 10 120 $B > $R/$O/c3_r3ref2.json 2> $R/$O/c3_r3ref2.err) || exit 1
JH_LIB=$V/libjh_tune.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_stream.json 2> $O/tl_stream.err || exit 1
JH_LIB=$V/libjh_p1legacy.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_stream_leg.json 2> $O/tl_stream_leg.err || exit 1
exit 0
