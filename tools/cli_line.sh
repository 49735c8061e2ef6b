# The product command's own rate: `katago selfplay` with a config for SECONDS on one GPU (a
# random-init b6c96 in a fresh models dir), then SIGTERM (rows flushed); its last stats lines.
#   bash tools/cli_line.sh CONFIG SECONDS   (e.g. configs/selfplay_coffee5.cfg 90)
set -u
cfg=$1; secs=$2
d=$(mktemp -d)
mkdir -p $d/models $d/out
python -c "import katacoffee_amd as kc; kc.write_random_model('b6c96', 0xC0FFEE, '$d/models/b6c96-s0.cfnn')" || exit 1
timeout -s TERM -k 20 $secs katacoffee_amd/katago selfplay -config $cfg -models-dir $d/models -output-dir $d/out > gpurun_out/cli_line.log 2>&1
rc=$?
grep -E "rows/s|audited" gpurun_out/cli_line.log | tail -8
echo "rows files: $(find $d/out -name '*.npz' | wc -l)"
rm -rf $d
# timeout's TERM is the expected end (rc 124)
[ $rc -eq 0 ] || [ $rc -eq 124 ]
