# C3 / C4 step under environment knobs. Each argument: workload:rank:VAR=v,VAR=v
# (rank ignored for c4; "-" for no variables).
#   gpurun -- bash tools/gpu_knob_sweep.sh <outdir> c3:0:JH_BFS_CUS=32 c3:3:JH_BFS_CUS=32 c4:0:-
O=${1:-gpurun_out/knobs}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p $O
for spec in "$@"; do
  IFS=: read W K VARS <<< "$spec"
  ENVS=""; [ "$VARS" != "-" ] && ENVS=$(echo $VARS | tr ',' ' ')
  STEPS=10; [ $W = c4 ] && STEPS=3
  env $ENVS timeout -k 10 300 python -u bench.py --workload $W --steps $STEPS --warmup 1 --no-cpu --no-parity --e2e 0 --seed-rank $K > "$O/$spec.log" 2>&1 || exit 1
  echo "$spec $(tail -1 "$O/$spec.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(round(d["ms_per_step"],2), round(c["phase1_ms"],2), round(c["phase2_seq_ms"],2), c["unknown_keys"])')" >> $O/sweep.txt
done
