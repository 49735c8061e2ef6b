# One rocprofv3 PMC pass (FETCH_SIZE or WRITE_SIZE, nothing else in the pass) over a
# bench.py command, reduced to per-kernel averages:
#   bash tools/prof_pmc.sh NAME COUNTER [bench.py args...]   (GPU box; gpu.sh run= step)
# No trace domains beside --pmc (the pool refuses them together).
set -u
name=$1
ctr=$2
shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 280 rocprofv3 --pmc $ctr -d gpurun_out/prof_$name -o $name --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line "$@" > gpurun_out/prof_$name.log 2>&1 || { echo "profiled run failed rc=$?"; tail -5 gpurun_out/prof_$name.log; exit 1; }
python tools/reduce_profile.py pmc gpurun_out/prof_$name $name
