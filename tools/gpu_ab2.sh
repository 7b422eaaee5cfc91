# round-5 A/B 2: the HBM-insert log for resume saves (variant log = bfs1 + log)
O=gpurun_out/r5ab2
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
JH_LIB=$R/jepsen_amd/variants/libjh_log.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lin.py -k "resume or stream or frontier or heavy or c3 or bfs" > $O/tests_log.log 2>&1 || exit 1
JH_TL_CSV=$R/$O/tl_r0.csv bash tools/gpu_r5.sh $O timeline tli "0" || exit 1
JH_TL_CSV=$R/$O/tl_r4.csv bash tools/gpu_r5.sh $O timeline tli "4" || exit 1
bash tools/gpu_r5.sh $O ab "0 4" 3 log bfs1
