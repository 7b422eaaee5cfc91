# round-5 A/B 3: phase 2's LEAN role at 8 / 12 waves per CU on phase-2-sized tables
O=gpurun_out/r5ab3
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
for v in p2w8 p2w12; do
  JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lin.py -k "resume or frontier or heavy or c3 or bfs or budget or phase" > $O/tests_$v.log 2>&1 || exit 1
done
bash tools/gpu_r5.sh $O ab "0 4 3" 2 cur p2w8 p2w12 || exit 1
JH_LIB=$R/jepsen_amd/variants/libjh_p2w8.so timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/c4_p2w8.json 2> $O/c4_p2w8.err || exit 1
JH_LIB=$R/jepsen_amd/variants/libjh_cur.so timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/c4_cur.json 2> $O/c4_cur.err
