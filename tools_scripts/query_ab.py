#!/usr/bin/env python3
"""Query-kernel A/B on the bench workload (1M-node synthetic graph, one
16384-row batch, 1M queries with targets in the batch): prints one JSON line
with q/s for the dense and RLE index under the CPD_TS_* knobs of this process.
The plan is cached in --cache (built on first use)."""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-oracle-search_amd"))
import numpy as np
import cpd

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1000)
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--queries", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--modes", default="dense,rle")
ap.add_argument("--cache", default="/tmp/cpd-bench-cache")
a = ap.parse_args()
os.makedirs(a.cache, exist_ok=True)
g = cpd.synth_road_graph(a.width, a.width, seed=a.seed)
plan, _ = cpd.Plan.cache(os.path.join(a.cache, f"synth{a.width}-s{a.seed}-ch823.plan"), g)
dev = cpd.Graph(plan, device=0)
owned = cpd.owned_nodes(g.n, 1, "div", 8, 0)
targets = owned[: dev.batch]
rows = dev.build_rows(targets)
rng = np.random.default_rng(100)
s = rng.integers(0, g.n, a.queries).astype(np.uint32)
t = targets[rng.integers(0, len(targets), a.queries)]
out = {"knobs": {k: v for k, v in os.environ.items() if k.startswith("CPD_TS")}}
for mode in a.modes.split(","):
    ix = cpd.Index(dev, rows=rows)
    ix.set_mode(mode)
    ix.prepare(s, t)
    ix.run()
    ms = []
    for _ in range(a.reps):
        ms.append(ix.run()["kernel_ms"])
    st = ix.run()
    out[mode] = {"qps": round(a.queries / (min(ms) / 1e3)), "ms_min": round(min(ms), 3),
                 "ms_med": round(sorted(ms)[len(ms) // 2], 3), "hops": st["hops"]}
    del ix
print(json.dumps(out), flush=True)
