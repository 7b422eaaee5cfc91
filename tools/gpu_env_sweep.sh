# C3 step under phase-2 knobs: each argument is late_us,helpers,quick[,rank].
#   gpurun -- bash tools/gpu_env_sweep.sh <outdir> 2000,16,8192 1000,32,8192,3 ...
O=${1:-gpurun_out/envsweep}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for cfg in "$@"; do
  IFS=, read L H Q K <<< "$cfg"
  JH_HELPER_LATE_US=$L JH_HELPERS=$H JH_QUICK_BUDGET=$Q timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-parity --e2e 0 --seed-rank ${K:-0} > $O/b_$cfg.log 2>&1 || exit 1
  echo "late=$L helpers=$H quick=$Q rank=${K:-0} $(tail -1 $O/b_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(round(d["ms_per_step"],2), round(c["phase1_ms"],2), round(c["phase2_seq_ms"],2))')" >> $O/sweep.txt
done
