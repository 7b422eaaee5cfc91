# round 5: packed host-buffer staging (jh_ingest.hip): its GPU tests, the
# host-buffer GPU tests, then C3 and C2 host-to-host A/B against plain copies
O=gpurun_out/r5ing
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_counter_set.py tests/test_gpu_ingest.py tests/test_c_harness.py > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --steps 5 --warmup 1 --no-cpu --no-parity"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c3_ing_$i.json 2> $O/c3_ing_$i.err || exit 1
  JH_INGEST_PLAIN=1 timeout -k 10 200 $B > $O/c3_plain_$i.json 2> $O/c3_plain_$i.err || exit 1
done
timeout -k 10 200 python -u tools/bench_c2.py --steps 3 --warmup 1 --no-cpu --e2e > $O/c2_ing.log 2>&1
JH_INGEST_PLAIN=1 timeout -k 10 200 python -u tools/bench_c2.py --steps 3 --warmup 1 --no-cpu --e2e > $O/c2_plain.log 2>&1
exit 0
