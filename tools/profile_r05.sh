# round-5 profiles (GPU box): rocprofv3 kernel traces of the bench lines and FETCH/WRITE
# PMC passes (one counter per pass, no trace domains beside --pmc), reduced in place by
# tools/reduce_profile.py.  Sections: bash tools/profile_r05.sh c2 corrected accurate c3 c4 c4pmc c2pmc
# Each GPU step has its own time limit; the first failing step ends the script.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
trace() {  # name, bench args...
  local name=$1
  shift
  run timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o $name --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line "$@" > gpurun_out/prof_$name.log 2>&1
  run python tools/reduce_profile.py trace gpurun_out/prof_$name $name
  grep '^{' gpurun_out/prof_$name.log > gpurun_out/prof_$name.line.json || true
}
pmc() {  # name, counter, bench args...
  local name=$1 ctr=$2
  shift 2
  run timeout -k 10 420 rocprofv3 --pmc $ctr -d gpurun_out/prof_$name -o $name --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line "$@" > gpurun_out/prof_$name.log 2>&1
  run python tools/reduce_profile.py pmc gpurun_out/prof_$name $name
}
nnpmc() {  # name, counter, nn_bench args... (the network alone; the C4 bench under --pmc
  # crashed inside the profiler's dispatch path, a host SIGSEGV in the launch call)
  local name=$1 ctr=$2
  shift 2
  run timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/prof_$name -o $name --output-format csv -- python tools/nn_bench.py "$@" > gpurun_out/prof_$name.log 2>&1
  run python tools/reduce_profile.py pmc gpurun_out/prof_$name $name
}
SHORT="--window short --warmup 8 --steps 6 --rounds-per-step 200"
for s in "$@"; do
  case $s in
    c2) trace r05_c2 --steps 20 --warmup 5 ;;
    corrected) trace r05_c2corr --steps 20 --warmup 5 --precision corrected ;;
    compliant) trace r05_c2default --steps 20 --warmup 5 --precision default ;;
    c3default) trace r05_c3default --config C3 --steps 10 --warmup 5 --precision default ;;
    accurate) trace r05_c2acc --steps 20 --warmup 5 --precision accurate ;;
    c3) trace r05_c3 --config C3 --steps 10 --warmup 5 ;;
    c4) trace r05_c4 --config C4 $SHORT ;;
    c5) trace r05_c5 --config C5 --window short --warmup 2 --steps 3 --rounds-per-step 600 ;;
    c4pmc)
      pmc r05_c4_fetch FETCH_SIZE --config C4 $SHORT
      pmc r05_c4_write WRITE_SIZE --config C4 $SHORT ;;
    c2pmc)
      pmc r05_c2_fetch FETCH_SIZE $SHORT
      pmc r05_c2_write WRITE_SIZE $SHORT ;;
    c4nn)
      nnpmc r05_c4nn_fetch FETCH_SIZE --arch b10c128 --board 7 --n 4096 --iters 5
      nnpmc r05_c4nn_write WRITE_SIZE --arch b10c128 --board 7 --n 4096 --iters 5 ;;
    c3nn)
      nnpmc r05_c3nn_fetch FETCH_SIZE --arch b10c128 --board 5 --n 4450 --iters 5
      nnpmc r05_c3nn_write WRITE_SIZE --arch b10c128 --board 5 --n 4450 --iters 5 ;;
    accpmc)
      pmc r05_c2acc_fetch FETCH_SIZE $SHORT --precision accurate
      pmc r05_c2acc_write WRITE_SIZE $SHORT --precision accurate ;;
    corrpmc)
      pmc r05_c2corr_fetch FETCH_SIZE $SHORT --precision corrected
      pmc r05_c2corr_write WRITE_SIZE $SHORT --precision corrected ;;
    lines34)
      run timeout -k 10 700 python -u bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/line_r05_c3.log 2>&1
      run timeout -k 10 440 python -u bench.py --config C4 --steps 6 --warmup 5 --no-cpu-baseline > gpurun_out/line_r05_c4.log 2>&1 ;;
    *) echo "unknown section $s"; exit 2 ;;
  esac
done
find gpurun_out/prof_r05_* -type f | head -60
