# GPU tests, then C2 bench lines at 1 and 2 game groups (each step time-limited;
# nothing further runs on the GPU after a failed step).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for g in ${GROUPS_LIST:-1 2}; do
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 20 --no-cpu-baseline --groups $g > gpurun_out/grp_$g.json 2> gpurun_out/grp_$g.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/grp_$g.json'))
print('groups $g rows/s %.0f playouts/s %.3g evals/s %.3g ms/step %.1f' % (d['value'], d['playouts_per_sec'], d['nn_evals_per_sec'], d['ms_per_step']), {n: round(v['avg_us'] or 0,1) for n,v in d['kernels'].items()})"
done
