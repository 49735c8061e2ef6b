# C3 / C4 at one and two game groups over full windows (30 steps after 10 warm-up).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in C3 C4; do
  for g in 1 2; do
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --config $c --groups $g --steps 30 --warmup 10 > gpurun_out/cg2_$c$g.json 2> gpurun_out/cg2_$c$g.err || { tail -3 gpurun_out/cg2_$c$g.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/cg2_$c$g.json'))
print('$c groups $g rows/s %.0f playouts/s %.3g ms/step %.2f' % (d['value'], d['playouts_per_sec'], d['ms_per_step']))"
  done
done
