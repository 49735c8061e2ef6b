# round-3 profiles: C2 bench + rocprofv3 kernel trace/stats of the same command, FETCH/WRITE
# PMC passes on a shorter window; C3 and C5 (layered network) traces.  Each GPU step time-limited.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
PA="--no-cpu-baseline"
MA="--no-cpu-baseline --warmup 16 --steps 8 --rounds-per-step 250"
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace --output-format csv -- python bench.py $PA > gpurun_out/prof_trace.log 2>&1
run python tools/reduce_profile.py trace gpurun_out/prof_trace trace
run timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o fetch --output-format csv -- python bench.py $MA > gpurun_out/prof_fetch.log 2>&1
run python tools/reduce_profile.py pmc gpurun_out/prof_fetch fetch
run timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o write --output-format csv -- python bench.py $MA > gpurun_out/prof_write.log 2>&1
run python tools/reduce_profile.py pmc gpurun_out/prof_write write
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 --output-format csv -- python bench.py --config C3 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1
run python tools/reduce_profile.py trace gpurun_out/prof_c3 c3
run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python bench.py --config C5 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1
run python tools/reduce_profile.py trace gpurun_out/prof_c5 c5
find gpurun_out/prof_* -type f | head -40
