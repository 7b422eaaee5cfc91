# A/B of a variant library on C3 (ranks 0/3), the C4 shard and C5.
#   gpurun -- bash tools/gpu_ab_workloads.sh <outdir> <variant>
O=${1:-gpurun_out/abw}; V=${2:-q7b}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for L in default $V; do
  if [ $L = default ]; then unset JH_LIB; else export JH_LIB=$R/jepsen_amd/variants/libjh_$L.so; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --e2e 0 > $O/${L}_c3.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --seed-rank 3 > $O/${L}_c3r3.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/${L}_c4.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu --e2e 0 > $O/${L}_c5.log 2>&1 || exit 1
done
