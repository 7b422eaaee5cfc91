# A/B of the heavy-pass CU split (BFS workgroups vs sequential waves)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bab
for b in "$@"; do
  JH_BFS_CUS=$b JH_DEBUG=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/bab/b$b.log 2>&1 || exit 1
done
