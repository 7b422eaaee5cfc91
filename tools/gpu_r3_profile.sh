# Round-3 evidence for profiles/r03: rocprofv3 kernel stats of the bench lines
# (C3 rank 0 and 3, C5, C2 counter + set) and FETCH_SIZE / WRITE_SIZE passes
# (one counter per pass) of the counter and set kernels and of the C3 search
# kernels.
#   gpurun --timeout 1200 -- bash tools/gpu_r3_profile.sh <outdir>
O=${1:-gpurun_out/r3prof}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
ks() {  # name, timeout, command...
  n=$1; t=$2; shift 2
  timeout -s KILL $t rocprofv3 --kernel-trace --stats -d $R/$O/$n -o $n --output-format csv -- "$@" > $R/$O/$n.log 2>&1
}
pmc() {  # name, counter, kernel regex, command...
  n=$1; c=$2; k=$3; shift 3
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "$k" -d $R/$O/pmc_$n -o $n --output-format csv -- "$@" > $R/$O/pmc_$n.log 2>&1
}
ks c3 300 python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity || exit 1
ks c3r3 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank 3 || exit 1
ks c2 300 python3 $R/tools/bench_c2.py --steps 3 --warmup 1 --no-cpu || exit 1
pmc c2_fetch FETCH_SIZE "k_cnt_|k_set_" python3 $R/tools/bench_c2.py --steps 1 --warmup 0 --no-cpu || exit 1
pmc c2_write WRITE_SIZE "k_cnt_|k_set_" python3 $R/tools/bench_c2.py --steps 1 --warmup 0 --no-cpu || exit 1
pmc c3_fetch FETCH_SIZE "k_lin_" python3 $R/tools/run_once.py c3 1 0 || exit 1
pmc c3_write WRITE_SIZE "k_lin_" python3 $R/tools/run_once.py c3 1 0 || exit 1
ks c5 400 python3 $R/bench.py --workload c5 --steps 1 --warmup 0 --no-cpu --e2e 0 --no-parity || exit 1
exit 0
