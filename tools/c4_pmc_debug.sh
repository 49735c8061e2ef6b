# C4 bench under rocprofv3 --pmc (the round-4 host SIGSEGV in launchSelect): the process map
# is dumped after the first warm-up step so a native stack's addresses can be resolved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KATACOFFEE_DUMP_MAPS=gpurun_out/c4pmc_maps.txt
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_c4dbg -o c4dbg --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line --config C4 --window short --warmup 8 --steps 6 --rounds-per-step 200 > gpurun_out/c4pmc_dbg.log 2>&1
rc=$?
echo "c4 pmc rc=$rc"
tail -5 gpurun_out/c4pmc_dbg.log
exit $rc
