# Same-box A/B of library variants on a short C4 bench window (default precision):
#   bash tools/ab_c4.sh VARIANT... (main = the in-tree library)
for v in "$@"; do
  if [ $v = main ]; then unset KATACOFFEE_LIB; else export KATACOFFEE_LIB=tools/_build/libkatacoffee_$v.so; fi
  timeout -k 10 300 python bench.py --config C4 --window short --warmup 6 --steps 4 --rounds-per-step 200 --no-cpu-baseline > gpurun_out/ab_c4_$v.$$.log 2>&1 || { echo "$v failed"; exit 1; }
  python - "$v" gpurun_out/ab_c4_$v.$$.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
k = d["kernels"]
print("%-8s %.0f moves/s  %.0f playouts/s  net %.1f us  select %.1f  backup %.1f" % (sys.argv[1], d["value"],
      d["playouts_per_sec"], k["network"]["avg_us"], k["select"]["avg_us"], k["backup"]["avg_us"]), flush=True)
PY
done
