#!/bin/bash
# One GPU session: parity tests, then (only if nothing crashed) a short bench.
# Exit codes 0/1 from pytest are test outcomes; anything else (abort, segfault,
# timeout) ends the session without further GPU work.
set -u
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "pytest crashed or timed out; stopping"
  exit $rc
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"
  tail -5 gpurun_out/bench.log
  exit $brc
fi
exit $rc
