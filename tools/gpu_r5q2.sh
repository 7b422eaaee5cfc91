# round 5 at HEAD, part 2: C4, C5, the C3 search kernels' FETCH / WRITE passes,
# and the host-buffer probe with the ingest trace
O=gpurun_out/r5q
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
JH_LIB=$R/jepsen_amd/variants/libjh_ingt.so JH_INGEST_TRACE=1 timeout -k 10 300 python -u tools/ingest_probe.py > $O/ingest_probe.log 2>&1 || exit 1
bash tools/gpu_r5.sh $O evidence2
