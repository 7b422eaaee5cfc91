# Round 4: C3 rank-0 A/B on one box -- round-3 build (git worktree r3ref/)
# against HEAD (block memo / legacy memo, streaming on / off), then the
# streaming timeline (JH_DEFER_TIMES, tuning builds).
#   gpurun --timeout 1200 -- bash tools/gpu_r4_ab3.sh <outdir>
O=${1:-gpurun_out/r4ab3}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
(cd $R/r3ref && timeout -k 10 120 $B > $R/$O/c3_r3ref.json 2> $R/$O/c3_r3ref.err) || exit 1
timeout -k 10 120 $B > $O/c3_head.json 2> $O/c3_head.err || exit 1
timeout -k 10 120 $B --opt flags=256 > $O/c3_head_ns.json 2> $O/c3_head_ns.err || exit 1
JH_LIB=$V/libjh_p1legacy.so timeout -k 10 120 $B --opt flags=256 > $O/c3_leg_ns.json 2> $O/c3_leg_ns.err || exit 1
JH_LIB=$V/libjh_p1legacy.so timeout -k 10 120 $B > $O/c3_leg.json 2> $O/c3_leg.err || exit 1
(cd $R/r3ref && timeout -k 10 120 $B > $R/$O/c3_r3ref2.json 2> $R/$O/c3_r3ref2.err) || exit 1
JH_LIB=$V/libjh_tune.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_stream.json 2> $O/tl_stream.err || exit 1
JH_LIB=$V/libjh_p1legacy_t.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity > $O/tl_stream_leg.json 2> $O/tl_stream_leg.err || exit 1
JH_LIB=$V/libjh_p1legacy_t.so JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity --opt flags=256 > $O/tl_ns_leg.json 2> $O/tl_ns_leg.err || exit 1
exit 0
