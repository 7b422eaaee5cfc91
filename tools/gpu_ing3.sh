O=gpurun_out/r5ing3
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
L=$R/jepsen_amd/variants/libjh_ingt.so
JH_LIB=$L JH_INGEST_TRACE=1 timeout -k 10 300 python -u tools/ingest_probe.py > $O/ing.log 2>&1 || exit 1
JH_LIB=$L JH_INGEST_PLAIN=1 timeout -k 10 300 python -u tools/ingest_probe.py > $O/plain.log 2>&1
