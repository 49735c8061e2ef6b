# search-kernel iteration: parity suite, then the phase profile (profiling build)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/t4.log 2>&1
rc=$?
tail -5 gpurun_out/t4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/search_phase.py --rounds 400 > gpurun_out/sphase.log 2>&1
rc=$?
cat gpurun_out/sphase.log
exit $rc
