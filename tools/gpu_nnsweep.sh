cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
t() { timeout -k 10 200 python -u tools/nn_bench.py "$@" || exit 1; }
t --arch b6c96 --n 2048,4096
t --arch b6c96 --precision fast-layered --n 512,2048,8192
t --arch b10c128 --precision fast --n 977,4096,16384
t --arch b10c128 --board 7 --n 600,4096
t --arch b18c384nbt --board 9 --n 484,4096 --iters 5
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nn -o nn --output-format csv -- python tools/nn_bench.py --arch b18c384nbt --board 9 --n 484 --iters 5 > gpurun_out/prof_nn.log 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/prof_nn/nn_kernel_stats.csv | head -12
