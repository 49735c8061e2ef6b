# GPU clock / power / temperature samples (rocm-smi, read-only) every 10 s while a bench
# line runs: does the sustained C4 window throttle?  Usage (GPU box):
#   bash tools/clock_watch.sh NAME LIMIT bench args...
name=$1; lim=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 $lim python -u bench.py "$@" > gpurun_out/clock_$name.log 2>&1 &
pid=$!
t0=$(date +%s)
while kill -0 $pid 2>/dev/null; do
  echo "== t=$(( $(date +%s) - t0 )) s" >> gpurun_out/clock_$name.smi
  rocm-smi --showclocks --showpower --showtemp >> gpurun_out/clock_$name.smi 2>&1
  sleep 10
done
wait $pid
rc=$?
echo "bench rc=$rc"
exit $rc
