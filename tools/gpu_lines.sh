# Bench lines beside the default C2 one: C2 with selfplay1.cfg play settings, C3, C4, C5
# (default groups per config).  Each GPU step time-limited; stop at the first failure.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  local n=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/line_$n.json 2> gpurun_out/line_$n.err || { tail -3 gpurun_out/line_$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/line_$n.json'))
print('$n rows/s %.0f playouts/s %.3g ms/step %.2f frac %.3f' % (d['value'], d['playouts_per_sec'], d['ms_per_step'], d['roofline']['frac']))"
}
run c2prod --play production --steps 60 --warmup 20
run c3 --config C3 --steps 30 --warmup 10
run c4 --config C4 --steps 30 --warmup 10
run c5 --config C5 --steps 50 --warmup 50
