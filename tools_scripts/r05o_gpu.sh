# synth4m: the step at the auto batch (with PMC) and at 4096 rows (fixed-latency fit for the compact up-store question)
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --workload synth4m --no-cpu --no-search --no-full-build > gpurun_out/r05o_4m.json 2> gpurun_out/r05o_4m.err || { tail -5 gpurun_out/r05o_4m.err; exit 1; }
cut -c1-250 gpurun_out/r05o_4m.json
timeout -k 10 600 python bench.py --workload synth4m --no-cpu --no-search --no-full-build --no-pmc --batch 4096 --queries 100000 > gpurun_out/r05o_4m_b4096.json 2> gpurun_out/r05o_4m_b4096.err || { tail -5 gpurun_out/r05o_4m_b4096.err; exit 1; }
cut -c1-250 gpurun_out/r05o_4m_b4096.json
