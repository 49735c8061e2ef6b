# round-2 GPU check: network paths (fused + layered, all BASELINE nets), trained net, parity
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_nn.py tests/test_gpu_train.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "exit $rc" >> gpurun_out/t1.log
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t1.log | tail -60
exit $rc
