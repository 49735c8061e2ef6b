# Round-structure experiments: a kernel trace of the default C2 bench, then bench lines
# over game groups x commit interval.  Each GPU step time-limited, stop at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/exp_trace -o trace --output-format csv -- python bench.py --no-cpu-baseline --steps 30 --warmup 20 > gpurun_out/exp_trace.log 2>&1 || exit 1
python tools/reduce_profile.py trace gpurun_out/exp_trace trace || exit 1
for cfg in "2 8" "2 16" "1 16"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 20 --no-cpu-baseline --groups $1 --commit-interval $2 > gpurun_out/exp_$1_$2.json 2> gpurun_out/exp_$1_$2.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/exp_$1_$2.json'))
print('groups $1 ci $2 rows/s %.0f playouts/s %.3g ms/step %.2f' % (d['value'], d['playouts_per_sec'], d['ms_per_step']), {n: round(v['avg_us'] or 0,1) for n,v in d['kernels'].items()})"
done
