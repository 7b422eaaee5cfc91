# A/B: heavy-key LDS Bloom 8 KB (default) vs 16 KB on rank 6 and rank 4 histories
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for r in 6 4; do
  JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-parity --e2e 0 --steps 3 --warmup 1 --seed-rank $r > gpurun_out/ab/base_r$r.log 2>&1 || exit 1
  JH_LIB=$GRAFT_REPO_ROOT/jepsen_amd/variants/libjh_bloom17.so JH_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --steps 3 --warmup 1 --seed-rank $r > gpurun_out/ab/b17_r$r.log 2>&1 || exit 1
done
