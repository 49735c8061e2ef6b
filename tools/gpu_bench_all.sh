# round-2: short bench lines for every config (no CPU leg), each under its own limit
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { name=$1; shift; echo "== $name: $*"; timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/b_$name.json 2> gpurun_out/b_$name.err; rc=$?; tail -c 600 gpurun_out/b_$name.json; echo; echo "rc=$rc"; return $rc; }
run C2 --steps 10 --warmup 5 && \
run C3 --config C3 --steps 5 --warmup 3 && \
run C4 --config C4 --steps 5 --warmup 3 && \
run C5 --config C5 --steps 3 --warmup 2 && \
run C2acc --precision accurate --steps 5 --warmup 3
