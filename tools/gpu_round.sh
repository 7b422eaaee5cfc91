# Round evidence at HEAD, one gpurun call: every -m gpu test, smoke, the C3
# bench line (parity + both CPU baselines), a rocprofv3 kernel-trace summary of
# the bench, and the phase-2 kernel's FETCH_SIZE / WRITE_SIZE passes.
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <outdir>
O=${1:-gpurun_out/round}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_c3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 > $R/$O/kt.log 2>&1 || exit 1
bash $R/tools/gpu_pmc.sh c3 "k_lin_seq<" $O/pmc_c3
