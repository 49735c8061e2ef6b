#!/bin/bash
# Bench + rocprofv3 kernel statistics + two PMC passes (FETCH_SIZE, WRITE_SIZE).
# The profiled passes run the same bench command as the bench line (default
# workload and window), so the rocprof per-kernel averages and the bench's live
# HIP-event averages describe the same launches.
# Every GPU step has its own time limit; any crash/timeout ends the session.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BA=${BENCH_ARGS:-""}
PA=${PROF_ARGS:-"--no-cpu-baseline $BA"}
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 ${BENCH_TIMEOUT:-500} python bench.py $BA > gpurun_out/bench.json 2> gpurun_out/bench.err
tail -c 3000 gpurun_out/bench.json
if [ -n "${NO_PROF:-}" ]; then exit 0; fi
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace --output-format csv -- python bench.py $PA > gpurun_out/prof_trace.log 2>&1
tail -c 1500 gpurun_out/prof_trace.log
if [ -n "${NO_PMC:-}" ]; then exit 0; fi
run timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o fetch --output-format csv -- python bench.py $PA > gpurun_out/prof_fetch.log 2>&1
run timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o write --output-format csv -- python bench.py $PA > gpurun_out/prof_write.log 2>&1
find gpurun_out -name "*.csv" | head -20
