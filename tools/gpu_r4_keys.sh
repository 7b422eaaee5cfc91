# Round 4: the critical C3 keys alone, per engine (tools/key_probe.py).
#   gpurun --timeout 900 -- bash tools/gpu_r4_keys.sh <outdir>
O=${1:-gpurun_out/r4keys}
R=$GRAFT_REPO_ROOT
V=$R/jepsen_amd/variants
cd $R && mkdir -p $O
export JH_LIB=$V/libjh_tune.so JH_DEBUG=2
timeout -k 10 200 python -u tools/key_probe.py c3 0 1086 > $O/k1086.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/key_probe.py c3 0 1086 8979 4457 8190 1342 5496 > $O/k6.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/key_probe.py c3 3 4136 > $O/k4136.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/key_probe.py c3 0 4031 > $O/k4031.log 2>&1 || exit 1
exit 0
