set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof_kt_bench.json 2> $R/gpurun_out/prof_kt_bench.err
echo kt-done
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --queries 100000 > $R/gpurun_out/prof_fetch_bench.json 2> $R/gpurun_out/prof_fetch.err
echo fetch-done
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --queries 100000 > $R/gpurun_out/prof_write_bench.json 2> $R/gpurun_out/prof_write.err
echo write-done
find $R/gpurun_out/prof_kt $R/gpurun_out/prof_fetch $R/gpurun_out/prof_write -name "*.csv" | head -20
