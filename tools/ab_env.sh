# Same-box A/B of environment settings on the C2 bench at one precision:
#   bash tools/ab_env.sh PRECISION 'VAR=VALUE ...' 'VAR=VALUE ...' ...   ('-' = no setting)
prec=$1; shift
i=0
for e in "$@"; do
  i=$((i + 1))
  envs=()
  [ "$e" != "-" ] && envs=($e)
  timeout -k 10 400 env "${envs[@]}" python bench.py --no-cpu-baseline --no-compliant-line --precision $prec \
    --steps 10 --warmup 5 > gpurun_out/ab_env_$i.log 2>&1 || { echo "$e failed"; exit 1; }
  python - "$e" gpurun_out/ab_env_$i.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
k = d["kernels"]
f = lambda nm: ("%.1f" % k[nm]["avg_us"]) if k.get(nm, {}).get("avg_us") else "-"
print("%-28s %.0f rows/s  net %s us  select %s  backup %s  backup+select %s" % (sys.argv[1], d["value"], f("network"),
      f("select"), f("backup"), f("backup_select")), flush=True)
PY
done
