# round-6 profiles and bench lines (GPU box): rocprofv3 kernel traces of bench lines,
# reduced in place by tools/reduce_profile.py, and the JSON lines of every config.
# Sections: bash tools/profile_r06.sh c2 c2default c3default c4default lines prodline
# Each GPU step has its own time limit; the first failing step ends the script.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# bench.py raises the HIP hardware-queue count itself, but under rocprofv3 the runtime may be
# initialised before bench.py's main runs: give the profiled process the same 8 queues
export GPU_MAX_HW_QUEUES=8
mkdir -p gpurun_out
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
trace() {  # name, bench args...
  local name=$1
  shift
  run timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o $name --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line --trained-steps 0 "$@" > gpurun_out/prof_$name.log 2>&1
  run python tools/reduce_profile.py trace gpurun_out/prof_$name $name
  grep '^{' gpurun_out/prof_$name.log > gpurun_out/prof_$name.line.json || true
}
pmcr() {  # name, counter, bench args...: counters only for the search kernels' dispatches
  # 3000-3399 of each (rounds ~1500-1700 of two game groups: past the first full-visit
  # searches, trees at their steady per-move size); every dispatch is still traced by the
  # profiler, so a crash in its dispatch path (profiles/r05/c4_pmc_crash.txt) still ends it
  local name=$1 ctr=$2
  shift 2
  run timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-include-regex "kSelect|kBackup|kCompact" --kernel-iteration-range "[3000-3399]" -d gpurun_out/prof_$name -o $name --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line --trained-steps 0 "$@" > gpurun_out/prof_$name.log 2>&1
  run python tools/reduce_profile.py pmc gpurun_out/prof_$name $name
}
pmc() {  # name, counter, bench args...: every dispatch of the short C2 window
  local name=$1 ctr=$2
  shift 2
  run timeout -k 10 420 rocprofv3 --pmc $ctr -d gpurun_out/prof_$name -o $name --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line --trained-steps 0 "$@" > gpurun_out/prof_$name.log 2>&1
  run python tools/reduce_profile.py pmc gpurun_out/prof_$name $name
}
SHORT="--window short --warmup 8 --steps 6 --rounds-per-step 200"
line() {  # name, limit, bench args...
  local name=$1 lim=$2
  shift 2
  run timeout -k 10 $lim python -u bench.py "$@" > gpurun_out/line_r06_$name.log 2>&1
  grep '^{' gpurun_out/line_r06_$name.log > gpurun_out/line_r06_$name.json || true
  echo "== line $name"
}
for s in "$@"; do
  case $s in
    c2) trace r06_c2 --steps 20 --warmup 5 ;;
    c2final) trace r06_c2final --steps 20 --warmup 5 ;;
    c2finaldefault) trace r06_c2finaldefault --steps 20 --warmup 5 --precision default ;;
    c2default) trace r06_c2default --steps 20 --warmup 5 --precision default ;;
    c3default) trace r06_c3default --config C3 --steps 10 --warmup 5 ;;
    c5default) trace r06_c5default --config C5 --window short --warmup 2 --steps 3 --rounds-per-step 100 ;;
    c4default) trace r06_c4default --config C4 --window short --warmup 8 --steps 6 --rounds-per-step 200 ;;
    c4pmc)
      pmcr r06_c4steady_fetch FETCH_SIZE --config C4 --window short --warmup 9 --steps 1 --rounds-per-step 200
      pmcr r06_c4steady_write WRITE_SIZE --config C4 --window short --warmup 9 --steps 1 --rounds-per-step 200 ;;
    c2pmc)
      pmc r06_c2_fetch FETCH_SIZE $SHORT
      pmc r06_c2_write WRITE_SIZE $SHORT ;;
    corrpmc)
      pmc r06_c2corr_fetch FETCH_SIZE $SHORT --precision corrected
      pmc r06_c2corr_write WRITE_SIZE $SHORT --precision corrected ;;
    accpmc)
      pmc r06_c2acc_fetch FETCH_SIZE $SHORT --precision accurate
      pmc r06_c2acc_write WRITE_SIZE $SHORT --precision accurate ;;
    main) line c2 600 --steps 20 --warmup 5 ;;
    prodline) line c2prod 600 --steps 20 --warmup 5 --play production --no-cpu-baseline --trained-steps 0 ;;
    c3line) line c3 700 --config C3 --steps 20 --warmup 5 --no-cpu-baseline ;;
    c4line) line c4 500 --config C4 --steps 6 --warmup 5 --no-cpu-baseline ;;
    c4g4line) line c4g4 500 --config C4 --steps 6 --warmup 5 --no-cpu-baseline --groups 4 ;;
    c3g4line) line c3g4 700 --config C3 --steps 20 --warmup 5 --no-cpu-baseline --groups 4 ;;
    c5line) line c5 500 --config C5 --steps 4 --warmup 2 --rounds-per-step 600 --no-cpu-baseline ;;
    *) echo "unknown section $s"; exit 2 ;;
  esac
done
find gpurun_out/prof_r06_* -type f 2>/dev/null | head -60
