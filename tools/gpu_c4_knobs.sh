# C4 shard under phase-2 / helper knobs (jh_lin_opts via --opt), default first
#   gpurun -- bash tools/gpu_c4_knobs.sh <outdir> "helpers=16" "phase2_budget=131072" ...
O=${1:-gpurun_out/c4knobs}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
B="python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity"
timeout -k 10 300 $B > $O/default.log 2>&1 || exit 1
for kv in "$@"; do
  timeout -k 10 300 $B --opt $kv > $O/$kv.log 2>&1 || exit 1
done
exit 0
