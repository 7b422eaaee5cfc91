# round 5: phase 2's LEAN memo / Bloom split, rank 0 at more repetitions and C4
O=gpurun_out/r5bl3
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
bash tools/gpu_r5.sh $O ab "0" 4 pb17 p9b17 || exit 1
for v in pb17 p9b17; do
  JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/c4_$v.json 2> $O/c4_$v.err || exit 1
done
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/c4_base.json 2> $O/c4_base.err
