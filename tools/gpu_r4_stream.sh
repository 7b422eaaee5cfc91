# Round 4: the streaming heavy-key pass against the round-3 schedule.
# Lin / counter parity tests, then C3 (rank 0, 3, 6) A/B lines (default =
# streamed, --opt flags=256 = JH_LIN_NO_STREAM), then the phase-1 traffic and
# DFS-stats passes of tools/gpu_r4_probe.sh.
#   gpurun --timeout 1200 -- bash tools/gpu_r4_stream.sh <outdir>
O=${1:-gpurun_out/r4stream}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_counter_set.py tests/test_c_harness.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for rk in 0 3 6; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --seed-rank $rk > $O/c3_r${rk}_stream.json 2> $O/c3_r${rk}_stream.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank $rk --opt flags=256 > $O/c3_r${rk}_legacy.json 2> $O/c3_r${rk}_legacy.err || exit 1
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu --e2e 0 > $O/c4_stream.json 2> $O/c4_stream.err || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu --e2e 0 > $O/c5_stream.json 2> $O/c5_stream.err || exit 1
exit 0
