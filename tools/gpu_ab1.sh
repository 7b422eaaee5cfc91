O=gpurun_out/r5ab1
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
JH_LIB=$R/jepsen_amd/variants/libjh_bfs1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lin.py -k "bfs or linear or frontier or heavy or c3 or configs or resume" > $O/tests_bfs1.log 2>&1 || exit 1
bash tools/gpu_r5.sh $O ab "0 4 3" 3 hbo bfs1 || exit 1
bash tools/gpu_r5.sh $O c2ab 3 cp0 cp2 cp3w6 || exit 1
bash tools/gpu_r5.sh $O timeline tlhbo "0"
