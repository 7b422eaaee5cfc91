O=gpurun_out/r5ing2
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py > $O/cs_ing.log 2>&1
JH_INGEST_PLAIN=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py > $O/cs_plain.log 2>&1
exit 0
