# Same-box A/B of bench.py argument sets (C2 unless an argument set says otherwise):
#   bash tools/ab_args.sh ARG:ARG:... ARG:... ...   (- = no extra arguments; ":" separates, so gpu.sh run= can pass sets)
i=0
for a in "$@"; do
  i=$((i + 1))
  extra=()
  [ "$a" != "-" ] && extra=(${a//:/ })
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-compliant-line --steps 10 --warmup 5 "${extra[@]}" \
    > gpurun_out/ab_args_$i.log 2>&1 || { echo "$a failed"; exit 1; }
  python - "$a" gpurun_out/ab_args_$i.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
k = d["kernels"]
f = lambda nm: ("%.1f" % k[nm]["avg_us"]) if k.get(nm, {}).get("avg_us") else "-"
print("%-40s %.0f rows/s  net %s us  select %s  backup %s  backup+select %s" % (sys.argv[1], d["value"], f("network"),
      f("select"), f("backup"), f("backup_select")), flush=True)
PY
done
