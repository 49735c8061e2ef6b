# A/B of two builds of libkatacoffee on the same box: alternating C2 bench runs
# (A = ab/libkatacoffee_head.so, B = the working tree's library).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export KATACOFFEE_LIB=$PWD/ab/libkatacoffee_head.so; else unset KATACOFFEE_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 60 --warmup 20 --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v$r.json'))
print('$v$r rows/s %.0f playouts/s %.3g ms/step %.2f' % (d['value'], d['playouts_per_sec'], d['ms_per_step']), {n: round(v['avg_us'] or 0,1) for n,v in d['kernels'].items()})"
  done
done
