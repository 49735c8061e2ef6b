#!/bin/bash
# rocprofv3 --pmc on minimal runs (tools/pmc_probe.py); PROBES = comma-separated
# argument lists; stops at the first crash.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IFS=',' read -ra LIST <<< "${PROBES:-fake 100 64,net 100 64,net 400 4096}"
for args in "${LIST[@]}"; do
  tag=$(echo $args | tr ' ' '_')
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/probe_$tag -o p --output-format csv -- python tools/pmc_probe.py $args > gpurun_out/probe_$tag.log 2>&1
  rc=$?
  echo "probe $args rc=$rc"
  grep -v "^\s*@" gpurun_out/probe_$tag.log | grep -v rocprofv3 | tail -2
  rm -rf gpurun_out/probe_$tag
  if [ $rc -ne 0 ]; then exit $rc; fi
done
