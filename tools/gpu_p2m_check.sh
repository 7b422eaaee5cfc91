cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/p2m
for M in 0 1; do
  JH_P2_M=$M timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu --no-parity --e2e 0 > gpurun_out/p2m/c5_$M.log 2>&1 || exit 1
done
JH_P2_M=1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 --seed-rank 6 > gpurun_out/p2m/r6_1.log 2>&1 || exit 1
