# Same-box A/B of library variants on the C2 bench at one precision:
#   bash tools/ab_bench.sh PRECISION VARIANT... (main = the in-tree library)
prec=$1; shift
for v in "$@"; do
  if [ $v = main ]; then unset KATACOFFEE_LIB; else export KATACOFFEE_LIB=tools/_build/libkatacoffee_$v.so; fi
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-compliant-line --precision $prec --steps 10 --warmup 5 --trained-steps 0 > gpurun_out/ab_bench_$v.$$.log 2>&1 || { echo "$v failed"; exit 1; }
  python - "$v" gpurun_out/ab_bench_$v.$$.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
k = d["kernels"]
print("%-8s %.0f rows/s  net %.1f us  select %.1f  backup %.1f" % (sys.argv[1], d["value"], k["network"]["avg_us"],
      k["select"]["avg_us"], k["backup"]["avg_us"]), flush=True)
PY
done
