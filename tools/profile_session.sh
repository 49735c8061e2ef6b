#!/bin/bash
# Bench + rocprofv3 kernel statistics + two PMC passes (FETCH_SIZE, WRITE_SIZE).
# The trace pass runs the same bench command as the bench line (default workload and
# window), so the rocprof per-kernel averages and the bench's live HIP-event averages
# describe the same launches.  The PMC passes use a shorter window in the same steady
# game-cycle phase mix, synchronised every 250 rounds (rocprofv3 --pmc segfaults in its
# dispatch hook once ~10k+ dispatches are queued without a host synchronisation).
# Large per-dispatch CSVs are reduced on the box (tools/reduce_profile.py).
# Every GPU step has its own time limit; any crash/timeout ends the session.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BA=${BENCH_ARGS:-""}
PA=${PROF_ARGS:-"--no-cpu-baseline $BA"}
MA=${PMC_ARGS:-"--no-cpu-baseline --warmup 16 --steps 8 --rounds-per-step 250"}
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
if [ -z "${NO_BENCH:-}" ]; then
  run timeout -k 10 ${BENCH_TIMEOUT:-500} python bench.py $BA > gpurun_out/bench.json 2> gpurun_out/bench.err
  tail -c 3000 gpurun_out/bench.json
fi
if [ -n "${NO_PROF:-}" ]; then exit 0; fi
if [ -z "${NO_TRACE:-}" ]; then
  run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace --output-format csv -- python bench.py $PA > gpurun_out/prof_trace.log 2>&1
  run python tools/reduce_profile.py trace gpurun_out/prof_trace trace
  tail -c 1500 gpurun_out/prof_trace.log
fi
if [ -n "${NO_PMC:-}" ]; then exit 0; fi
run timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o fetch --output-format csv -- python bench.py $MA > gpurun_out/prof_fetch.log 2>&1
run python tools/reduce_profile.py pmc gpurun_out/prof_fetch fetch
run timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o write --output-format csv -- python bench.py $MA > gpurun_out/prof_write.log 2>&1
run python tools/reduce_profile.py pmc gpurun_out/prof_write write
find gpurun_out -name "*.csv" -o -name "*.json" | head -20
