# The one GPU-box driver script: `gpurun -- bash tools/gpu.sh STEP [STEP ...]`.
# Steps run in order, each under its own time limit; the first failing step ends the
# call (no further GPU work after a fault, abort or timeout).  Logs go to gpurun_out/.
#   test[=PATTERN]   pytest -m gpu (optionally -k PATTERN)
#   file=PATH        pytest of one test file (gpu-marked tests in it)
#   bench[=ARGS]     python bench.py ARGS (comma-separated: bench=--config,C3,--steps,10)
#   benchlong[=ARGS] the same with a 1050 s limit (long-game windows: C5 rows on disk)
#   lines            tools/bench_lines.sh (every config's bench line, gpurun_out/lines.json)
#   smoke            __graft_entry__.smoke()
#   prof             tools/profile_r03.sh (rocprofv3 trace + PMC passes)
#   prof4=SECTIONS   tools/profile_r04.sh (comma-separated sections: prof4=c2,corrected,c4,c4pmc)
#   prof5=SECTIONS   tools/profile_r05.sh (the same sections named r05_*, plus compliant, c3default, lines34)
#   prof6=SECTIONS   tools/profile_r06.sh (traces c2, c2default, c3default, c4default; lines main, prodline,
#                    c3line, c4line, c5line)
#   run=CMD          any other command (comma-separated words), e.g. run=tools/_build/nn_phase,960
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  log=gpurun_out/step${n}_${name}.log
  case $name in
    test)
      k=()
      [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread "${k[@]}" > $log 2>&1 ;;
    file)
      timeout -k 10 900 python -u -m pytest "$arg" -m gpu -x -v -rP --timeout 300 --timeout-method thread > $log 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg//,/ } > $log 2>&1 ;;
    benchlong)
      timeout -k 10 1050 python -u bench.py ${arg//,/ } > $log 2>&1 ;;
    lines)
      timeout -k 10 1100 bash tools/bench_lines.sh > $log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
    run)
      timeout -k 10 300 ${arg//,/ } > $log 2>&1 ;;
    prof)
      timeout -k 10 1100 bash tools/profile_r03.sh > $log 2>&1 ;;
    prof4)
      timeout -k 10 1100 bash tools/profile_r04.sh ${arg//,/ } > $log 2>&1 ;;
    prof5)
      timeout -k 10 1150 bash tools/profile_r05.sh ${arg//,/ } > $log 2>&1 ;;
    prof6)
      timeout -k 10 1150 bash tools/profile_r06.sh ${arg//,/ } > $log 2>&1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "== step $n $step rc=$rc"
  grep -E "PASSED|FAILED|ERROR|passed|failed|smoke ok|Error|error" $log | tail -40
  tail -c 1500 $log | tail -3
  [ $rc -eq 0 ] || exit $rc
done
