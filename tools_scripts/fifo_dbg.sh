# fifo_auto on a fresh 3-worker index: one request through the FIFO protocol
mkdir -p gpurun_out/dbg && cd gpurun_out/dbg || exit 1
../../bin/gen_synth --width 30 --height 24 --seed 2 --out g --queries 3000 > /dev/null || exit 1
for w in 0 1 2; do timeout -k 5 60 ../../bin/make_cpd_auto --input g.xy --partmethod mod --partkey 3 --workerid $w --maxworker 3 --outdir idx --device 0 > mk$w.log 2>&1 || { echo "make_cpd_auto $w failed"; cat mk$w.log; exit 1; }; done
F=$PWD/w0.fifo; rm -f $F
timeout -k 5 60 ../../bin/fifo_auto --input g.xy g.xy.diff --partmethod mod --partkey 3 --workerid 0 --maxworker 3 --outdir idx --alg table-search --device 0 --fifo $F --once > fa.log 2>&1 &
P=$!
for i in $(seq 1 60); do grep -q listening fa.log && break; sleep 0.5; done
echo "--- fa.log after wait"; cat fa.log
printf '3\n0 3\n4 6\n7 9\n' > q.txt
rm -f ans.fifo; mkfifo ans.fifo
printf '{"hscale": 1.0, "debug": true}\n%s %s -\n' $PWD/q.txt $PWD/ans.fifo > $F &
timeout 20 cat ans.fifo; echo "cat rc=$?"
wait $P; echo "fifo_auto rc=$?"
echo "--- fa.log"; cat fa.log; cat q.txt.res
