# End-of-round evidence: profiles (tools/profile_r02.sh), then the default bench line
# with its CPU legs.  Stops at the first failed step.
cd "$GRAFT_REPO_ROOT"
bash tools/profile_r02.sh > gpurun_out/profile_session.log 2>&1 || { tail -5 gpurun_out/profile_session.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
tail -c 600 gpurun_out/bench_default.json
