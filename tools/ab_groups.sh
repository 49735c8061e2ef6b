# Same-box C2 bench over game-group counts and HIP hardware-queue limits (GPU_MAX_HW_QUEUES,
# the HIP runtime's streams-to-hardware-queues mapping; 4 by default):
#   bash tools/ab_groups.sh PRECISION "GROUPS:QUEUES" ...   e.g. default 2:4 4:4 4:8
# (BENCH_ARGS: other bench.py arguments, default "--steps 10 --warmup 5")
prec=$1; shift
for gq in "$@"; do
  g=${gq%%:*}; q=${gq##*:}
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --no-compliant-line --trained-steps 0 --precision $prec --groups $g ${BENCH_ARGS:---steps 10 --warmup 5} > gpurun_out/ab_groups_${g}_${q}.$$.log 2>&1 || { echo "$gq failed"; exit 1; }
  python - "$gq" gpurun_out/ab_groups_${g}_${q}.$$.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
k = d["kernels"]
print("groups:queues %-5s %.0f rows/s  %.2f M playouts/s  net %.1f us  select %s  backup %s  backup_select %s" % (
      sys.argv[1], d["value"], d["playouts_per_sec"] / 1e6, k["network"]["avg_us"], k["select"]["avg_us"],
      k["backup"]["avg_us"], k["backup_select"]["avg_us"]), flush=True)
PY
done
