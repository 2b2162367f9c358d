# full GPU suite, then the fscale-0 search leg A/B: lane-major vs array-major workspaces
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r05c_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/r05c_gputest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05c_gputest.log | head; exit $rc; }
for lm in 1 0; do CPD_SEARCH_LANE_MAJOR=$lm CPD_SEARCH_TRACE=1 timeout -k 10 400 python bench.py --no-cpu --no-full-build --no-pmc --steps 5 > gpurun_out/r05c_lm$lm.json 2> gpurun_out/r05c_lm$lm.err || { tail -5 gpurun_out/r05c_lm$lm.err; exit 1; }; done
echo done
