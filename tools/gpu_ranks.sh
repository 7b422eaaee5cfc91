# C3 lines of the ranks the other scripts do not run (seed 3 + 7919 r), for the 8-GPU picture
#   gpurun -- bash tools/gpu_ranks.sh
O=gpurun_out/ranks
mkdir -p $O
for rk in 1 2 4 5 7; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank $rk > $O/r$rk.log 2>&1 || exit 1
done
exit 0
