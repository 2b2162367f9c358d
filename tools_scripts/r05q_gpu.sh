# counters of the search kernel at fscale 0 (what bounds it)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/r05q_counters.txt 2>&1 || true
timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 --queries 16384 > gpurun_out/r05q_warm.json 2> gpurun_out/r05q_warm.err || { tail -5 gpurun_out/r05q_warm.err; exit 1; }
cat gpurun_out/r05q_warm.json | cut -c1-300
timeout -k 10 1000 python tools_scripts/search_pmc.py gpurun_out/r05q_search_pmc.json --fscale 0 --queries 16384
