# round 5: the cost of phase 1's memo writes -- a -DJH_DUP_WRITE build writes
# every HBM memo insert twice (a 16 B scattered store into an unread 1 GB
# mirror); phase 1's time against the release build, and its WRITE_SIZE
O=gpurun_out/r5p/dup
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p $O
bash tools/gpu_r5.sh $O ab "0 4" 3 dup || exit 1
cd /tmp && export TMPDIR=/tmp
JH_LIB=$R/jepsen_amd/variants/libjh_dup.so timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_lin_dfs -d $R/$O/pmc_dup/write -o write --output-format csv -- python3 $R/tools/run_once.py c3 1 0 > $R/$O/pmc_dup_write.log 2>&1
