# round-2: C2 bench lines: default (with CPU baseline), the driver's short window, a long window, production
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { name=$1; shift; echo "== $name: $*"; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/c2_$name.json 2> gpurun_out/c2_$name.err; rc=$?; echo "rc=$rc"; return $rc; }
run driver --steps 20 --warmup 5 --no-cpu-baseline && \
run long --steps 150 --warmup 30 --no-cpu-baseline && \
run prod --play production --no-cpu-baseline && \
run default
