# round-5 bench lines of the other workloads on the current tree
mkdir -p gpurun_out
for w in melb300k synth1m-spec synth4m; do
  timeout -k 10 900 python bench.py --workload $w > gpurun_out/r05ad_bench_$w.json 2> gpurun_out/r05ad_bench_$w.err || { echo "$w failed"; tail -5 gpurun_out/r05ad_bench_$w.err; exit 1; }
  echo "$w $(cut -c1-220 gpurun_out/r05ad_bench_$w.json)"
done
