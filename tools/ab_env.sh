# Same-box A/B of environment switches on the C2 bench (alternating, REPS passes):
#   REPS=2 bash tools/ab_env.sh PRECISION NAME:VAR=VAL[,VAR=VAL] ...   (NAME: = no override)
# e.g. bash tools/ab_env.sh fast main: sep:COFFEE_SEPARATE_RESOLVE=1
prec=$1; shift
reps=${REPS:-2}
for r in $(seq $reps); do
  for v in "$@"; do
    name=${v%%:*}
    envs=${v#*:}
    log=gpurun_out/ab_env_${name}_$r.$$.log
    env ${envs//,/ } timeout -k 10 400 python bench.py --no-cpu-baseline --no-compliant-line --precision $prec \
      --steps 10 --warmup 5 --trained-steps 0 > $log 2>&1 || { echo "$name failed"; exit 1; }
    python - "$name" $log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
k = d["kernels"]
f = lambda n: k[n]["avg_us"] or 0.0
print("%-8s %.0f rows/s  net %.1f us  select %.1f  backup %.1f  backup_select %.1f" % (
    sys.argv[1], d["value"], f("network"), f("select"), f("backup"), f("backup_select")), flush=True)
PY
  done
done
