# One rocprofv3 kernel trace (+ stats) of a bench.py command, reduced to per-kernel
# averages: bash tools/prof_one.sh NAME [bench.py args...]  (GPU box; gpu.sh run= step)
set -u
name=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 280 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o $name --output-format csv -- python bench.py --no-cpu-baseline --no-compliant-line "$@" > gpurun_out/prof_$name.log 2>&1 || { echo "profiled run failed rc=$?"; tail -5 gpurun_out/prof_$name.log; exit 1; }
python tools/reduce_profile.py trace gpurun_out/prof_$name $name
