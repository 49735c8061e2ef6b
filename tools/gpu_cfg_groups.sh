# C2 (current kCompact) and C3-C5 bench lines at one and two game groups.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/cg_$n.json 2> gpurun_out/cg_$n.err || { tail -3 gpurun_out/cg_$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/cg_$n.json'))
print('$n rows/s %.0f playouts/s %.3g ms/step %.2f' % (d['value'], d['playouts_per_sec'], d['ms_per_step']), {k: round(v['avg_us'] or 0,1) for k,v in d['kernels'].items()})"
}
run c2g2 --steps 60 --warmup 20
for c in C3 C4 C5; do
  for g in 1 2; do
    run ${c}g$g --config $c --groups $g --steps 10 --warmup 5
  done
done
