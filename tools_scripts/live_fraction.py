#!/usr/bin/env python3
"""Offline estimate of how sparse the upward sweep is (host only, no GPU).

For a batch of targets split into slabs, d_up(x, t) is finite only for x in
t's upward search space (nodes that reach t along down-arcs).  This counts, per
up-level >= 2 (the materialised levels), the share of (node, slab) pairs with
at least one finite value — the rows the up-sweep must store — for slabs of
consecutive targets and for slabs sorted by DFS column.

  python tools_scripts/live_fraction.py [--width 1000] [--batch 16384] [--slab 1024]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-oracle-search_amd"))
import cpd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--slab", type=int, default=1024)
    ap.add_argument("--plan", default="/tmp/cpd-bench-cache/synth1000-s1-ch823.plan")
    a = ap.parse_args()
    g = cpd.synth_road_graph(a.width, a.width, seed=a.seed)
    if os.path.exists(a.plan):
        plan = cpd.Plan.load(a.plan)
    else:
        t0 = time.time()
        plan = cpd.Plan(g)
        os.makedirs(os.path.dirname(a.plan), exist_ok=True)
        plan.save(a.plan)
        print(f"plan built in {time.time() - t0:.1f}s", flush=True)
    ch = plan.export_ch()
    n = g.n
    lu = ch["level_up"]
    order = plan.order()
    # reverse of the down arcs: v -> x for every down-arc x -> v
    dn_off = ch["dn_off"].astype(np.int64)
    tails = np.repeat(np.arange(n, dtype=np.int64), np.diff(dn_off))
    heads = ch["dn_dst"].astype(np.int64)
    idx = np.argsort(heads, kind="stable")
    r_src = tails[idx]
    r_off = np.zeros(n + 1, np.int64)
    np.add.at(r_off, heads + 1, 1)
    r_off = np.cumsum(r_off)

    def reach(targets):
        seen = np.zeros(n, bool)
        seen[targets] = True
        front = np.unique(targets)
        while len(front):
            lo, hi = r_off[front], r_off[front + 1]
            cnt = hi - lo
            if cnt.sum() == 0:
                break
            rep = np.repeat(lo - np.cumsum(np.concatenate(([0], cnt[:-1]))), cnt)
            nb = r_src[np.arange(cnt.sum()) + rep]
            nb = np.unique(nb[~seen[nb]])
            seen[nb] = True
            front = nb
        return seen

    owned = cpd.owned_nodes(n, 1, "div", 8, 0)
    batch = owned[: a.batch]
    mat = lu >= 2
    nl = int(lu.max()) + 1
    per_level_nodes = np.bincount(lu[mat], minlength=nl)
    for label, tg in (("node-id order", batch), ("DFS-column sorted", batch[np.argsort(order[batch])])):
        live = np.zeros(nl)
        for s in range(0, len(tg), a.slab):
            seen = reach(tg[s:s + a.slab])
            live += np.bincount(lu[seen & mat], minlength=nl)
        slabs = len(tg) // a.slab
        tot = per_level_nodes.sum() * slabs
        print(f"{label}: live (node, slab) share over levels >= 2: {live.sum() / tot:.4f} "
              f"({int(live.sum())} of {tot})")
        for lv in list(range(2, min(nl, 12))) + list(range(12, nl, 20)):
            if per_level_nodes[lv]:
                print(f"  level {lv:3d}: nodes {per_level_nodes[lv]:7d} live "
                      f"{live[lv] / (per_level_nodes[lv] * slabs):.3f}")


if __name__ == "__main__":
    main()
