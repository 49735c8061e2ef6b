# GPU check after search changes: the self-play parity suite (incl. tree positions)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/t3.log 2>&1
rc=$?
echo "exit $rc" >> gpurun_out/t3.log
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t3.log | tail -60
exit $rc
