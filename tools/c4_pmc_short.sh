# C4 FETCH/WRITE PMC passes with a short run (rounds 5): the full C4 bench command crashed
# inside librocprofiler-sdk during the second warm-up step (profiles/r05/c4_pmc_crash.txt);
# this checks whether a run with fewer dispatches completes -- one warm-up step and one
# timed step of 100 rounds (the per-dispatch averages need no steady window).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-compliant-line --config C4 --window short --warmup 1 --steps 1 --rounds-per-step 100"
for ctr in FETCH_SIZE WRITE_SIZE; do
  n=r05_c4short_$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
  timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/prof_$n -o $n --output-format csv -- $B > gpurun_out/prof_$n.log 2>&1
  rc=$?
  echo "c4 short pmc $ctr: rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python tools/reduce_profile.py pmc gpurun_out/prof_$n $n || exit 1
done
