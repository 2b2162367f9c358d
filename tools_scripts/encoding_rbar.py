#!/usr/bin/env python3
"""Runs per row (R̄) of the CPD under alternative move encodings (DESIGN §2,
VERDICT r02 item 6).  Analysis only, CPU: the oracle's first-move sets and
greedy RLE (oracle/cpd_oracle.c) on a small synthetic road graph.

  E0 reverse CPD, move = index of the edge in the COLUMN node's own
     out-list (file order) — what libcpd and the oracle restate [U];
  E1 reverse CPD, move = the edge's compass direction (8 sectors of its
     dx, dy): one alphabet for every node, so neighbouring columns that head
     the same way share a symbol;
  E2 reverse CPD, move = the rank of the edge by angle to the straight line
     towards the row's target (0 = the edge pointing most directly at t);
  E3 forward CPD (warthog graph_oracle: row = source s, column = target in
     DFS order, move = index in s's out-list): the alphabet is one node's
     own edges for the whole row.

  python tools_scripts/encoding_rbar.py [--width 100] [--rows 48]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "distributed-oracle-search_amd"), os.path.join(ROOT, "oracle")]
import cpd  # noqa: E402
import oracle  # noqa: E402
from scipy.sparse import csr_matrix  # noqa: E402
from scipy.sparse.csgraph import dijkstra  # noqa: E402


def remap(fm, row_ptr, sym):
    """Map each node's edge-index set to a set over `sym[e]` (bit per symbol)."""
    out = np.empty_like(fm)
    for v in range(len(fm)):
        f = int(fm[v])
        if f == 0xFFFF:
            out[v] = 0xFFFF
            continue
        m = 0
        for k in range(row_ptr[v + 1] - row_ptr[v]):
            if f >> k & 1:
                m |= 1 << int(sym[row_ptr[v] + k])
        out[v] = m
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=100)
    ap.add_argument("--rows", type=int, default=48)
    a = ap.parse_args()
    res = {}
    for style in ("spec", "shuffled"):
        g = cpd.synth_road_graph(a.width, a.width, seed=1, style=style)
        n = g.n
        order = oracle.dfs_preorder(g.row_ptr, g.dst)
        src = np.repeat(np.arange(n), np.diff(g.row_ptr.astype(np.int64)))
        dx = (g.x[g.dst] - g.x[src]).astype(np.float64)
        dy = (g.y[g.dst] - g.y[src]).astype(np.float64)
        ang = np.arctan2(dy, dx)
        compass = (np.round(ang / (math.pi / 4)).astype(np.int64) % 8)
        rng = np.random.default_rng(3)
        rows = rng.choice(n, a.rows, replace=False)
        A = csr_matrix((g.w.astype(np.float64), g.dst, g.row_ptr), shape=(n, n))
        r = {"E0": [], "E1": [], "E2": [], "E3": []}
        for t in rows:
            fm = oracle.first_moves(g.row_ptr, g.dst, g.w, int(t))
            r["E0"].append(len(oracle.rle_row(fm, order)))
            r["E1"].append(len(oracle.rle_row(remap(fm, g.row_ptr, compass), order)))
            # E2: per node, its edges ranked by angle to the direction of t
            tx, ty = float(g.x[t]), float(g.y[t])
            rank = np.zeros(len(g.dst), np.int64)
            for v in range(n):
                e0, e1 = int(g.row_ptr[v]), int(g.row_ptr[v + 1])
                if e1 == e0:
                    continue
                want = math.atan2(ty - g.y[v], tx - g.x[v])
                dev = np.abs((ang[e0:e1] - want + math.pi) % (2 * math.pi) - math.pi)
                rank[e0 + np.argsort(dev, kind="stable")] = np.arange(e1 - e0)
            r["E2"].append(len(oracle.rle_row(remap(fm, g.row_ptr, rank), order)))
            # E3: forward row of source s = t: sets over s's own out-edges
            s = int(t)
            nb = g.dst[g.row_ptr[s]:g.row_ptr[s + 1]]
            ws = g.w[g.row_ptr[s]:g.row_ptr[s + 1]].astype(np.float64)
            D = dijkstra(A, indices=np.concatenate([[s], nb]))
            ds, dn = D[0], D[1:]
            f = np.zeros(n, np.uint16)
            for k in range(len(nb)):
                f |= (np.isclose(dn[k] + ws[k], ds) & np.isfinite(ds)).astype(np.uint16) << k
            f[~np.isfinite(ds)] = 0xFFFF
            f[s] = 0xFFFF
            r["E3"].append(len(oracle.rle_row(f, order)))
        res[style] = {"n": n, "rows": len(rows),
                      **{k: {"mean_runs": round(float(np.mean(v)), 1),
                             "per_n": round(float(np.mean(v)) / n, 4)} for k, v in r.items()}}
        print(style, json.dumps(res[style]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
