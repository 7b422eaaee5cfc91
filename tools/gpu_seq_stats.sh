# Per-wave statistics of the heavy-key sequential search (JH_DFS_STATS build)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
JH_LIB=jepsen_amd/variants/libjh_stats.so JH_DEBUG=2 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu --no-parity > gpurun_out/seq_stats.log 2>&1
