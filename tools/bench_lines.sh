# Bench lines of every BASELINE config on one GPU box (gpu.sh run= step or directly):
# C2 fast (the driver's default command: CPU baseline and the corrected-precision
# "compliant" window included), C2 accurate, C3, C4, C5.
# Each run is time-limited; the JSON lines are collected into gpurun_out/lines.json.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  name=$1
  shift
  timeout -k 10 420 python -u bench.py "$@" > gpurun_out/line_$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run c2 --steps 20 --warmup 5
run c2acc --steps 20 --warmup 5 --precision accurate --no-cpu-baseline
run c3 --config C3 --steps 20 --warmup 5 --no-cpu-baseline
run c4 --config C4 --steps 6 --warmup 5 --no-cpu-baseline
run c5 --config C5 --steps 4 --warmup 2 --rounds-per-step 600 --no-cpu-baseline
python - <<'EOF'
import json
out = {}
for n in ["c2", "c2acc", "c3", "c4", "c5"]:
    for line in open("gpurun_out/line_%s.log" % n):
        if line.startswith('{"metric"'):
            out[n] = json.loads(line)
json.dump(out, open("gpurun_out/lines.json", "w"), indent=1)
print({n: round(d["value"], 1) for n, d in out.items()})
EOF
