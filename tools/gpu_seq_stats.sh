# Per-wave statistics of the heavy-key sequential search (JH_DFS_STATS build), ranks 0 and 6
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ss
for r in 0 6; do
JH_LIB=jepsen_amd/variants/libjh_stats.so JH_DEBUG=2 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --no-parity --e2e 0 --seed-rank $r > gpurun_out/ss/r$r.log 2>&1 || exit 1
done
