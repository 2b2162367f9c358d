#!/usr/bin/env python3
"""Time the GPU contraction (verbose phase breakdown on stderr) of the
synthetic graph of side W (default 1000: configs[3]); --host also times the
host build.  python tools_scripts/ch_gpu_time.py [W] [--host]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-oracle-search_amd"))
import cpd  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1000
g = cpd.synth_road_graph(W, W, seed=1)
for rep in range(2):
    t = time.time()
    p = cpd.Plan(g, gpu=0, verbose=2 if rep == 0 else 1)  # 2: every round
    print(f"GPU plan {time.time() - t:.2f} s, CH {p.info()['ch_seconds']:.2f} s", flush=True)
if "--host" in sys.argv:
    t = time.time()
    p = cpd.Plan(g)
    print(f"host plan {time.time() - t:.2f} s, CH {p.info()['ch_seconds']:.2f} s", flush=True)
