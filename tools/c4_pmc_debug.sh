# C4 bench under rocprofv3 --pmc (rounds 4 and 5: a host SIGSEGV inside the profiler's
# dispatch interception, librocprofiler-sdk.so.1.1.0+0x1e72fb, during the second warm-up
# step -- in a kSelect<4> launch, and with kSelect excluded from counting in a layered
# conv launch).  Bisect on the number of streams: one game group (one HIP stream / HSA
# queue) instead of two.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KATACOFFEE_DUMP_MAPS=gpurun_out/c4pmc_maps.txt
B="python bench.py --no-cpu-baseline --no-compliant-line --config C4 --window short --warmup 8 --steps 6 --rounds-per-step 200"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_r05_c4g1_fetch -o r05_c4g1_fetch --output-format csv -- $B --groups 1 > gpurun_out/c4pmc_g1.log 2>&1
rc=$?
echo "c4 pmc, one game group: rc=$rc"
exit $rc
