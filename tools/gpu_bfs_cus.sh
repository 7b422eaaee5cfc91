# Sweep of the heavy-key CU split (BFS workgroups vs sequential waves) on C3.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 32 64 96 128; do
  JH_BFS_CUS=$c JH_DEBUG=1 timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu --no-parity > gpurun_out/bfs_cus_$c.log 2>&1 || exit 1
done
