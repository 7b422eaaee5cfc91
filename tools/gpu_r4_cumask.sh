# Round 4: the streamed heavy-key pass on CU-masked streams (tuning build,
# JH_CU_SPLIT=R: phase 1 on n_cu - R CUs, the consumers on R CUs from the
# start) against the default schedule and the unmasked streamed pass; C3 rank 0.
#   gpurun --timeout 900 -- bash tools/gpu_r4_cumask.sh <outdir>
O=${1:-gpurun_out/r4cumask}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
export JH_LIB=$V/libjh_tune.so
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
timeout -k 10 120 $B > $O/c3_default.json 2> $O/c3_default.err || exit 1
timeout -k 10 120 $B --opt flags=256 > $O/c3_stream.json 2> $O/c3_stream.err || exit 1
JH_CU_SPLIT=64 JH_BFS_CUS=16 JH_EARLY_LEAN=64 timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --opt flags=256 --opt helpers=16 > $O/c3_s64.json 2> $O/c3_s64.err || exit 1
JH_CU_SPLIT=96 JH_BFS_CUS=24 JH_EARLY_LEAN=96 timeout -k 10 120 $B --opt flags=256 --opt helpers=32 > $O/c3_s96.json 2> $O/c3_s96.err || exit 1
JH_CU_SPLIT=48 JH_BFS_CUS=12 JH_EARLY_LEAN=48 timeout -k 10 120 $B --opt flags=256 --opt helpers=12 > $O/c3_s48.json 2> $O/c3_s48.err || exit 1
JH_CU_SPLIT=128 JH_BFS_CUS=32 JH_EARLY_LEAN=128 timeout -k 10 120 $B --opt flags=256 --opt helpers=32 > $O/c3_s128.json 2> $O/c3_s128.err || exit 1
timeout -k 10 120 $B > $O/c3_default2.json 2> $O/c3_default2.err || exit 1
exit 0
