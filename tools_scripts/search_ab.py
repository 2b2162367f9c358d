#!/usr/bin/env python3
"""CPD-search A/B on the bench's search workload (1M-node synthetic graph, a
256-row dense index, the .diff stand-in weights, 65536 queries): one JSON
line with q/s and the pass trace for the knobs of this process
(CPD_SEARCH_*; --fscale, --capacity, --frac).  The plan is cached in --cache
(the bench's PLAN_TAG name)."""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-oracle-search_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import cpd
import bench

ap = argparse.ArgumentParser()
ap.add_argument("--fscale", type=float, default=0.0)
ap.add_argument("--queries", type=int, default=65536)
ap.add_argument("--capacity", type=int, default=0)
ap.add_argument("--capacity-max", type=int, default=0)
ap.add_argument("--frac", type=float, default=0.0)
ap.add_argument("--tables", default="auto")
ap.add_argument("--cache", default="/tmp/cpd-bench-cache")
a = ap.parse_args()
args = bench.parse(["--cache", a.cache])
os.makedirs(a.cache, exist_ok=True)
g = cpd.synth_road_graph(args.width, args.width, seed=args.seed, style=args.style)
pp = bench.plan_path(args)
if not os.path.exists(pp):
    cpd.Plan(g, gpu=0).save(pp)
plan = cpd.Plan.load(pp)
dev = cpd.Graph(plan, device=0, batch=1024)
dev.set_coords(g.x, g.y)
owned = bench.rank_targets(args, g.n, 1, 0)
srows = owned[:256]
rows = dev.build_rows(srows)
ix = cpd.Index.streamed(dev, srows, rows.count()[1], mode="dense")
ix.append_rows(rows)
del rows
ix.set_weights(cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3))
rng = np.random.default_rng(5)
s = rng.integers(0, g.n, a.queries).astype(np.uint32)
t = srows[rng.integers(0, len(srows), a.queries)]
ix.search(s[:64], t[:64], fscale=a.fscale, tables=a.tables)  # warm (tables built)
t0 = time.time()
_, _, fin, cnt, st = ix.search(s, t, fscale=a.fscale, capacity=a.capacity,
                               capacity_max=a.capacity_max, workspace_frac=a.frac,
                               tables=a.tables)
wall = time.time() - t0
print(json.dumps({"knobs": {k: v for k, v in os.environ.items() if k.startswith("CPD_SEARCH")},
                  "fscale": a.fscale, "capacity_arg": a.capacity, "frac": a.frac,
                  "qps": round(a.queries / (st["kernel_ms"] / 1e3), 1), "wall_s": round(wall, 3),
                  "expanded": int(st["expanded"]), "finished": int(fin.sum()),
                  **{k: st[k] for k in ("kernel_ms", "lanes", "passes", "capacity",
                                        "capacity_last", "resumed", "restarted", "overflow")}}),
      flush=True)
