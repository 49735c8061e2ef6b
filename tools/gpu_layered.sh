# layered-network check: GPU network tests, then C3 / C5 / accurate C2 bench lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nn.py -q --timeout 300 --timeout-method thread > gpurun_out/tnn.log 2>&1 || { tail -30 gpurun_out/tnn.log; exit 1; }
tail -2 gpurun_out/tnn.log
for c in C3 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/L_$c.json 2> gpurun_out/L_$c.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/L_$c.json')); n=d['roofline_all']['network']
print('$c rows/s %.0f playouts/s %.3g evals/s %.3g net %.0f us/launch %.0f evals %.0f TF frac %.3f' % (d['value'], d['playouts_per_sec'], d['nn_evals_per_sec'], n['avg_launch_us'], n['evals_per_launch'], n['achieved'], n['frac']))"
done
