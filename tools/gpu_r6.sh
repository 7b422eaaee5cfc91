# Round 6 GPU runs (round 5 script carried forward), one parameterised script (replaces round 4's one-off A/Bs):
#   gpurun --timeout T -- bash tools/gpu_r5.sh <outdir> <part> [args...]
# parts:
#   tests  <pytest args...>   GPU tests (e.g. tests/test_gpu_lin.py -k configs)
#   final                     the whole GPU suite, smoke(), the default bench line,
#                             the C3 kernel trace (rocprofv3 --kernel-trace --stats)
#   bench  <name> <bench.py args...>   one bench line -> <outdir>/<name>.json
#   ranks  [bench.py args...] C3 ranks 1-7 (--seed-rank) at 5 steps
#   prof   <name> <cmd...>    rocprofv3 kernel trace + stats of one command
#   pmc    <name> <counters> <cmd...>  one rocprofv3 --pmc pass
#   evidence / evidence2      the round's remaining evidence at HEAD (see below)
#   ab "<ranks>" <reps> <v>...  alternating C3 lines, in-tree build vs variants
#   abopt "<ranks>" <reps> <name>=<bench options>...  the same for jh_lin_opts
#   c2ab <reps> <v>...        counter parity tests + alternating C2 lines
#   tests_v <v> <pytest args...>   GPU tests on variants/libjh_<v>.so
#   pmc_v <v> <name> <counter> <kernel-regex> [workload]  a --pmc pass on a variant
#   c4 <name> [v]             the C4 line (on a variant)
#   c2 <name>                 the C2 lines with host-to-host timings
#   abenv <v> "<ranks>" <reps> <name>=<VAR=v,...>...  a -DJH_TUNING variant's JH_* knobs
#   ingest <v>                host-buffer calls, packed vs plain (a -DJH_TUNING variant)
#   timeline <v> "<ranks>"    per-key timeline of a -DJH_TUNING variant
# Variants are tools/build_variants.sh builds in jepsen_amd/variants/ (git-ignored).
# Round 5's runs as calls of this script (the profiles/r05/ directories they made):
#   ab_helpers_bfs   tests_v bfs1 tests/test_gpu_lin.py -k "bfs or linear or frontier or heavy or c3 or configs or resume"
#                    && ab "0 4 3" 3 hbo bfs1 && c2ab 3 cp0 cp2 cp3w6 && timeline tlhbo 0
#   ab_rs_log        tests_v log tests/test_gpu_lin.py -k "resume or stream or frontier or heavy or c3 or bfs"
#                    && timeline tli 0 && timeline tli 4 (JH_TL_CSV=<file>) && ab "0 4" 3 log bfs1
#   ab_p2_waves      tests_v p2w8 ... && tests_v p2w12 ... && ab "0 4 3" 2 cur p2w8 p2w12 && c4 p2w8 p2w8 && c4 cur cur
#   ab_p2_bloom      ab "0 4 3" 2 pb17 p9b17; ab "4 0 7" 2 pb17 pb18 p9b18; ab 0 4 pb17 p9b17 && c4 ...
#   ab_dup_write     ab "0 4" 3 dup && pmc_v dup pmc_dup WRITE_SIZE k_lin_dfs
#   ab_cnt_*         c2ab 3 <v>;   ab_bfs_claim  ab "4 3 0" 2 cl8
#   ab_helpers_r5q   abopt "0 4" 3 l2000h48="--opt helper_late_us=2000 --opt helpers=48" l3000h64="..."
#   ingest           tests_v - tests/test_gpu_configs.py tests/test_gpu_counter_set.py tests/test_gpu_ingest.py && ingest ingt
#   final_r5p / r5q  final && c2 bench_c2 && ranks && evidence2
O=${1:-gpurun_out/r5}; PART=${2:-final}; shift 2
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
case $PART in
tests)
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $O/tests.log 2>&1 ;;
final)
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || exit 1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c3prof -o c3 -- python3 $R/bench.py --steps 5 --warmup 0 --no-cpu --e2e 0 --no-parity > $R/$O/c3prof.log 2>&1 ;;
bench)
  N=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > $O/$N.json 2> $O/$N.err ;;
ranks)
  for rk in 1 2 3 4 5 6 7; do
    timeout -k 10 120 python -u bench.py --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1 --seed-rank $rk "$@" > $O/c3r${rk}.json 2> $O/c3r${rk}.err || exit 1
  done ;;
prof)
  N=$1; shift
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$N -o $N -- "$@" > $R/$O/$N.log 2>&1 ;;
pmc)
  N=$1; C=$2; shift 2
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/$O/$N -o $N -- "$@" > $R/$O/$N.log 2>&1 ;;
evidence)
  # the rest of the round's evidence at HEAD, part 1: C3 ranks 1-7, the
  # one-rank RCCL path, the C2 lines under a kernel trace
  for rk in 1 2 3 4 5 6 7; do
    timeout -k 10 120 python -u bench.py --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}.json 2> $O/c3r${rk}.err || exit 1
  done
  JH_BENCH_DIST1=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --pool 1 > $O/dist1.json 2> $O/dist1.err || exit 1
  JH_BENCH_DIST1=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 > $O/dist1_pool0.json 2> $O/dist1_pool0.err || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2prof -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 > $R/$O/bench_c2.log 2>&1 ;;
evidence2)
  # part 2: C4, C5, and the C3 search kernels' FETCH_SIZE / WRITE_SIZE passes
  # (tools/pmc_traffic.py on the CPU side)
  timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
  timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
  bash tools/gpu_pmc.sh c3 'k_lin_seq_lw' $O/pmc_c3 0 && bash tools/gpu_pmc.sh c3 'k_lin_dfs' $O/pmc_c3p1 0 ;;
ab)
  # alternating C3 runs of the in-tree build and of variants/libjh_<v>.so
  #   ab "<ranks>" <reps> <v>...
  RK=$1; REPS=$2; shift 2
  B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
  for i in $(seq 1 $REPS); do
    for rk in $RK; do
      timeout -k 10 120 $B --seed-rank $rk > $O/base_r${rk}_$i.json 2> $O/base_r${rk}_$i.err || exit 1
      for v in "$@"; do
        JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 120 $B --seed-rank $rk > $O/${v}_r${rk}_$i.json 2> $O/${v}_r${rk}_$i.err || exit 1
      done
    done
  done ;;
c2ab)
  # counter builds: each variant's counter parity tests, then alternating
  # C2 lines of the in-tree build and the variants: c2ab <reps> <v>...
  REPS=$1; shift
  for v in "$@"; do
    JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_counter_set.py tests/test_gpu_configs.py -k "counter or c2" > $O/tests_$v.log 2>&1 || exit 1
  done
  for i in $(seq 1 $REPS); do
    timeout -k 10 120 python -u tools/bench_c2.py --steps 10 --warmup 2 --no-cpu > $O/base_$i.log 2>&1 || exit 1
    for v in "$@"; do
      JH_LIB=$R/jepsen_amd/variants/libjh_$v.so timeout -k 10 120 python -u tools/bench_c2.py --steps 10 --warmup 2 --no-cpu > $O/${v}_$i.log 2>&1 || exit 1
    done
  done ;;
timeline)
  # per-key timeline of a -DJH_TUNING variant: timeline <v> "<ranks>"
  V=$1; RK=$2
  for rk in $RK; do
    JH_LIB=$R/jepsen_amd/variants/libjh_$V.so JH_DEBUG=1 JH_DEFER_TIMES=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank $rk > $O/tl_${V}_r$rk.log 2>&1 || exit 1
  done ;;
abopt)
  RK=$1; REPS=$2; shift 2
  B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
  for i in $(seq 1 $REPS); do
    for rk in $RK; do
      timeout -k 10 120 $B --seed-rank $rk > $O/ctl_r${rk}_$i.json 2>/dev/null || exit 1
      for nv in "$@"; do
        timeout -k 10 120 $B --seed-rank $rk ${nv#*=} > $O/${nv%%=*}_r${rk}_$i.json 2>/dev/null || exit 1
      done
    done
  done ;;
abshard)
  # alternating c3s shard lines (strong scaling), control vs jh_lin_opts variants:
  # abshard "<r/N>..." <reps> <name>=<bench options>...
  SH=$1; REPS=$2; shift 2
  B="python -u bench.py --workload c3s --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
  for i in $(seq 1 $REPS); do
    for sh in $SH; do
      t=${sh/\//of}
      timeout -k 10 150 $B --shard $sh > $O/ctl_s${t}_$i.json 2>/dev/null || exit 1
      for nv in "$@"; do
        timeout -k 10 150 $B --shard $sh ${nv#*=} > $O/${nv%%=*}_s${t}_$i.json 2>/dev/null || exit 1
      done
    done
  done ;;
tests_v)
  V=$1; shift
  L=""; [ "$V" != "-" ] && L=$R/jepsen_amd/variants/libjh_$V.so
  JH_LIB=$L timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $O/tests_$V.log 2>&1 ;;
pmc_v)
  V=$1; N=$2; C=$3; K=$4; W=${5:-c3}
  cd /tmp && export TMPDIR=/tmp
  JH_LIB=$R/jepsen_amd/variants/libjh_$V.so timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$K" -d $R/$O/$N -o $N --output-format csv -- python3 $R/tools/run_once.py $W 1 0 > $R/$O/$N.log 2>&1 ;;
c4)
  N=$1; V=$2
  L=""; [ -n "$V" ] && L=$R/jepsen_amd/variants/libjh_$V.so
  JH_LIB=$L timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e 0 > $O/c4_$N.json 2> $O/c4_$N.err ;;
c2)
  timeout -k 10 200 python -u tools/bench_c2.py --steps 5 --warmup 1 --e2e > $O/$1.log 2>&1 ;;
abenv)
  # a -DJH_TUNING variant under environment settings (its JH_* knobs):
  #   abenv <v> "<ranks>" <reps> <name>=<VAR=value,...>...
  V=$1; RK=$2; REPS=$3; shift 3
  B="python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
  for i in $(seq 1 $REPS); do
    for rk in $RK; do
      timeout -k 10 120 $B --seed-rank $rk > $O/base_r${rk}_$i.json 2>/dev/null || exit 1
      for nv in "$@"; do
        env $(echo ${nv#*=} | tr ',' ' ') JH_LIB=$R/jepsen_amd/variants/libjh_$V.so timeout -k 10 120 $B --seed-rank $rk > $O/${nv%%=*}_r${rk}_$i.json 2>/dev/null || exit 1
      done
    done
  done ;;
abenvsh)
  # abenv over c3s shards (strong scaling): abenvsh <v> "<r/N>..." <reps> <name>=<VAR=value,...>...
  V=$1; SH=$2; REPS=$3; shift 3
  B="python -u bench.py --workload c3s --steps 5 --warmup 1 --no-cpu --e2e 0 --no-parity"
  for i in $(seq 1 $REPS); do
    for sh in $SH; do
      t=${sh/\//of}
      timeout -k 10 150 $B --shard $sh > $O/base_s${t}_$i.json 2>/dev/null || exit 1
      for nv in "$@"; do
        env $(echo ${nv#*=} | tr ',' ' ') JH_LIB=$R/jepsen_amd/variants/libjh_$V.so timeout -k 10 150 $B --shard $sh > $O/${nv%%=*}_s${t}_$i.json 2>/dev/null || exit 1
      done
    done
  done ;;
ingest)
  L=$R/jepsen_amd/variants/libjh_$1.so
  JH_LIB=$L JH_INGEST_TRACE=1 timeout -k 10 300 python -u tools/ingest_probe.py > $O/ingest_packed.log 2>&1 || exit 1
  JH_LIB=$L JH_INGEST_PLAIN=1 timeout -k 10 300 python -u tools/ingest_probe.py > $O/ingest_plain.log 2>&1 ;;
probe)
  # per-key engine traces on a -DJH_TUNING variant: probe <v> "<env VAR=v,...>" <rank> <key>...
  V=$1; E=$2; RK=$3; shift 3
  env $(echo $E | tr ',' ' ') JH_LIB=$R/jepsen_amd/variants/libjh_$V.so timeout -k 10 150 python -u tools/key_probe.py c3 $RK "$@" > $O/probe_${V}_r${RK}_$(echo $E | tr ',=' '__').log 2>&1 ;;
strong)
  # C3 strong scaling (one 10k-key history split by key): every shard of N = 2, 4, 8 on this GPU
  for n in 2 4 8; do
    for rk in $(seq 0 $((n - 1))); do
      timeout -k 10 150 python -u bench.py --workload c3s --shard $rk/$n --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1 "$@" > $O/c3s_${rk}of${n}.json 2> $O/c3s_${rk}of${n}.err || exit 1
    done
  done ;;
rprobe)
  # per-key engine runs on the release library: rprobe <name> <rank> <key>... (JH_PROBE_FLAGS from the caller)
  N=$1; RK=$2; shift 2
  timeout -k 10 150 python -u tools/key_probe.py c3 $RK "$@" > $O/rprobe_$N.log 2>&1 ;;
tl)
  # per-key timeline CSV (JH_TL_CSV) of a -DJH_TUNING variant: tl <v> <name> <rank> [bench.py args...]
  V=$1; N=$2; RK=$3; shift 3
  JH_LIB=$R/jepsen_amd/variants/libjh_$V.so JH_DEFER_TIMES=1 JH_TL_CSV=$R/$O/tl_$N.csv timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e 0 --no-parity --seed-rank $RK "$@" > $O/tl_$N.json 2> $O/tl_$N.err ;;
ev6a)
  # round 6 evidence, part a: C3 strong-scaling shards (N = 2, 4, 8), ranks 1-7, the
  # C3 line at round 4's definition (budget 2^20, exact counts)
  for n in 2 4 8; do
    for rk in $(seq 0 $((n - 1))); do
      timeout -k 10 150 python -u bench.py --workload c3s --shard $rk/$n --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1 > $O/c3s_${rk}of${n}.json 2> $O/c3s_${rk}of${n}.err || exit 1
    done
  done
  for rk in 1 2 3 4 5 6 7; do
    timeout -k 10 120 python -u bench.py --no-cpu --e2e 0 --no-parity --steps 5 --warmup 1 --seed-rank $rk > $O/c3r${rk}.json 2> $O/c3r${rk}.err || exit 1
  done
  timeout -k 10 300 python -u bench.py --no-cpu --e2e 0 --steps 10 --warmup 2 --budget 1048576 --opt flags=1024 > $O/c3_r4def.json 2> $O/c3_r4def.err ;;
ev6b)
  # part b: C4, C5, C2 under a kernel trace, the one-rank RCCL path
  timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
  timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
  JH_BENCH_DIST1=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --steps 5 --warmup 1 --no-cpu --e2e 0 > $O/dist1_pool0.json 2> $O/dist1_pool0.err || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c2prof -o c2 -- python3 $R/tools/bench_c2.py --steps 5 --warmup 1 --e2e > $R/$O/bench_c2.log 2>&1 ;;
pmc6)
  # FETCH_SIZE / WRITE_SIZE passes over the C3 search kernels (tools/pmc_traffic.py on the CPU side)
  bash tools/gpu_pmc.sh c3 'k_lin_seq_lw' $O/pmc_c3 0 && bash tools/gpu_pmc.sh c3 'k_lin_dfs' $O/pmc_c3p1 0 ;;
ev6c)
  # part c: the PMC traffic passes, the C3 kernel trace at --warmup 0 (its
  # stats average = the line's timed launches), per-context HBM, k_cnt_pack's
  # instruction mix
  bash tools/gpu_pmc.sh c3 'k_lin_seq_lw' $O/pmc_c3 0 && bash tools/gpu_pmc.sh c3 'k_lin_dfs' $O/pmc_c3p1 0 || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c3prof -o c3 -- python3 $R/bench.py --steps 5 --warmup 0 --no-cpu --e2e 0 --no-parity > $R/$O/c3prof.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex k_cnt_pack --output-format csv -d $R/$O/cntsq -o cntsq -- python3 $R/tools/bench_c2.py --steps 1 --warmup 0 --no-cpu > $R/$O/cntsq.log 2>&1 || exit 1
  cd $R
  timeout -k 10 200 python -u tools/mem_probe.py 1 > $O/mem1.json 2> $O/mem1.err && timeout -k 10 200 python -u tools/mem_probe.py 2 > $O/mem2.json 2> $O/mem2.err ;;
*) echo "unknown part $PART"; exit 2 ;;
esac
