# C3 phase timings (two runs) and the C2 counter/set lines + kernel summary
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
JH_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 > gpurun_out/c3_run$i.log 2>&1 || exit 1
done
bash tools/gpu_c2.sh
