#!/usr/bin/env python3
"""A/B: one build workspace of B rows per step vs K workspaces (cpd_graph
objects, each with its own stream and buffers) of B/K rows built concurrently
from K host threads (ctypes releases the GIL inside libcpd), on the bench's
synth1m workload.  Prints one JSON line per configuration.

  python tools_scripts/workspaces_ab.py [--steps 10] [--configs 1x16384,2x8192,1x8192]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-oracle-search_amd"))

import bench  # noqa: E402
import cpd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--configs", default="1x16384,2x8192,1x8192")
    a = ap.parse_args()
    args = bench.parse(["--no-cpu", "--no-pmc"])
    os.makedirs(args.cache, exist_ok=True)
    g = cpd.synth_road_graph(args.width, args.width, seed=args.seed, style=args.style)
    plan, _ = cpd.Plan.cache(bench.plan_path(args), g)
    owned = bench.rank_targets(args, g.n, 1, 0)
    for cfg in a.configs.split(","):
        k, b = (int(v) for v in cfg.split("x"))
        devs = [cpd.Graph(plan, device=0, batch=b) for _ in range(k)]
        for d in devs:
            d.set_coords(g.x, g.y)
        rows = [None] * k

        def work(i, step):
            rows[i] = devs[i].build_rows(bench.batch_of(owned, b, step * k + i), reuse=rows[i])

        def step(s):
            ts = [threading.Thread(target=work, args=(i, s)) for i in range(k)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()

        step(0)
        step(1)
        t0 = time.perf_counter()
        for s in range(a.steps):
            step(2 + s)
        for r in rows:
            r.export_range(0, 1)  # waits for the last emit
        dt = time.perf_counter() - t0
        print(json.dumps({"workspaces": k, "batch": b, "steps": a.steps,
                          "rows_per_s": round(k * b * a.steps / dt, 1),
                          "ms_per_step": round(dt / a.steps * 1e3, 3)}), flush=True)
        del rows, devs


if __name__ == "__main__":
    main()
