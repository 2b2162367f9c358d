"""Seeded test graphs shared by the CPU and GPU suites."""
import numpy as np

import cpd


def graph_from_edges(n, edges):
    """edges: list of (a, b, w) in file order."""
    rp = np.zeros(n + 1, np.uint32)
    for a, _, _ in edges:
        rp[a + 1] += 1
    rp = np.cumsum(rp).astype(np.uint32)
    pos = rp[:-1].copy()
    dst = np.zeros(len(edges), np.uint32)
    w = np.zeros(len(edges), np.uint32)
    for a, b, c in edges:
        dst[pos[a]] = b
        w[pos[a]] = c
        pos[a] += 1
    return cpd.RoadGraph(rp, dst, w)


def irregular_graph():
    """Unreachable pairs, a degree-15 node, a self loop, parallel and 0-weight edges."""
    rng = np.random.default_rng(5)
    n = 300
    edges = []
    for a in range(n):
        k = 15 if a == 17 else int(rng.integers(0, 5))
        for _ in range(k):
            b = int(rng.integers(0, n))
            edges.append((a, b, int(rng.integers(0, 4))))
    edges.append((3, 3, 1))        # self loop
    edges.append((5, 9, 2))        # parallel edge pair
    edges.append((5, 9, 1))
    edges = [e for e in edges if not (e[1] >= 290)]   # nodes 290.. are never entered
    return graph_from_edges(n, edges)


def deg8_graph():
    """Out-degrees 5..8 on a ring (8-bit first-move sets), weights 1..3 (ties)."""
    rng = np.random.default_rng(8)
    n = 400
    edges = []
    for a in range(n):
        edges.append((a, (a + 1) % n, int(rng.integers(1, 4))))   # strongly connected ring
        for _ in range(int(rng.integers(4, 8))):
            edges.append((a, int(rng.integers(0, n)), int(rng.integers(1, 4))))
    return graph_from_edges(n, edges)


def ring2_graph():
    """Out-degree <= 2 (a two-way ring with a few chords removed: 2-slot
    adjacency, the shift-1 kernels), weights 1..5."""
    rng = np.random.default_rng(2)
    n = 500
    edges = []
    for a in range(n):
        edges.append((a, (a + 1) % n, int(rng.integers(1, 6))))
        if a % 7:
            edges.append((a, (a - 1) % n, int(rng.integers(1, 6))))
    return graph_from_edges(n, edges)


def tie_graph():
    """Tiny weights -> many equal-cost paths (multi-bit first-move sets)."""
    g = cpd.synth_road_graph(24, 24, seed=11)
    return cpd.RoadGraph(g.row_ptr, g.dst, (g.w % 3 + 1).astype(np.uint32), g.x, g.y)


GRAPHS = {
    "synth": lambda: cpd.synth_road_graph(40, 30, seed=7),
    "ties": tie_graph,
    "irregular": irregular_graph,
    "deg8": deg8_graph,
    "ring2": ring2_graph,
    "single": lambda: graph_from_edges(1, []),
}
