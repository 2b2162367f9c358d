"""Shared set-up of the at-size GPU tests (BASELINE.json configs): the graphs,
a per-session plan cache, and the sampled-target definition of configs[4]."""
import os

import numpy as np

import cpd

CACHE = os.environ.get("CPD_TEST_CACHE", "/tmp/cpd-test-cache")


def plan_for(g, tag):
    """The graph's plan, built once and cached on local disk for the session
    (and later sessions on the same box); its hierarchy contracted on GPU 0
    (ch_gpu.cpp: the host build's hierarchy, arc for arc — tests/test_ch_gpu.py)."""
    os.makedirs(CACHE, exist_ok=True)
    plan, _ = cpd.Plan.cache(os.path.join(CACHE, f"{tag}.plan"), g, gpu=0)
    return plan


def sample_targets(n, k, seed):
    """configs[4]: k targets sampled without replacement."""
    return np.sort(np.random.default_rng(seed).choice(n, size=k, replace=False)).astype(np.uint32)


def owned(nodes, maxworker, method, key, wid, n):
    """The members of `nodes` that worker `wid` owns (distribution_controller)."""
    nodes = np.asarray(nodes, np.int64)
    if method == "mod":
        bid = nodes % key
    else:
        bid = nodes // (-(-n // key))
    return nodes[(bid % maxworker) == wid].astype(np.uint32)


def spread(a, k):
    """k entries of a, evenly spaced (first and last included)."""
    idx = np.unique(np.linspace(0, len(a) - 1, k).round().astype(np.int64))
    return np.asarray(a)[idx]


def check_row_format(off, runs, n):
    """Every row starts at column 0, its run columns strictly increase and are
    < n; moves are 4-bit (checked by construction)."""
    off = np.asarray(off, np.int64)
    cols = (np.asarray(runs) >> 4).astype(np.int64)
    starts = off[:-1]
    assert np.all(np.diff(off) > 0)
    assert np.all(cols[starts] == 0)
    inc = np.diff(cols) > 0
    inc[starts[1:] - 1] = True  # row boundaries
    assert np.all(inc)
    assert cols.max() < n


def move_run_counts(mv, n, bits, chunk=1024):
    """Runs per row of compact rows (cpd_rows_export_moves layout), counted
    on the whole array in numpy: 1 (column 0) + the columns 1..n-1 whose move
    differs from the left neighbour's — the greedy RLE row's run count
    (DESIGN §2), so it must equal the row's offsets difference."""
    mv = np.ascontiguousarray(mv, np.uint32)
    per, W = 32 // bits, mv.shape[1]
    low = np.uint32(sum(1 << (bits * i) for i in range(per)))
    # per word: the fields of columns 1..n-1 (column 0 and pad never count)
    cols = np.arange(W * per, dtype=np.int64).reshape(W, per)
    ok = (cols >= 1) & (cols < n)
    valid = (ok.astype(np.uint64) << (bits * np.arange(per, dtype=np.uint64))).sum(axis=1)
    valid = valid.astype(np.uint32) & low
    out = np.empty(len(mv), np.int64)
    for a in range(0, len(mv), chunk):
        x = mv[a:a + chunk]
        carry = np.zeros_like(x)
        carry[:, 1:] = x[:, :-1] >> np.uint32(32 - bits)
        d = x ^ ((x << np.uint32(bits)) | carry)  # field c: move(c) ^ move(c-1)
        f = d
        for k in range(1, bits):
            f = f | (d >> np.uint32(k))
        out[a:a + chunk] = 1 + np.bitwise_count(f & valid).sum(axis=1, dtype=np.int64)
    return out


def hilbert_keys(x, y):
    """libcpd's lane key (cpd_gpu.cpp hilbert_keys): the Hilbert index of each
    node's coordinates on a 2^16 x 2^16 grid over the bounding box."""
    x = np.asarray(x, np.int64)
    y = np.asarray(y, np.int64)
    side = 1 << 16
    x0, y0 = x.min(), y.min()
    ext = max(x.max() - x0, y.max() - y0) + 1
    px = (x - x0) * (side - 1) // ext
    py = (y - y0) * (side - 1) // ext
    d = np.zeros(len(x), np.int64)
    s = side // 2
    while s > 0:
        rx = ((px & s) != 0).astype(np.int64)
        ry = ((py & s) != 0).astype(np.int64)
        d += s * s * ((3 * rx) ^ ry)
        rot = ry == 0
        flip = rot & (rx == 1)
        px = np.where(flip, side - 1 - px, px)
        py = np.where(flip, side - 1 - py, py)
        px, py = np.where(rot, py, px), np.where(rot, px, py)
        s //= 2
    return (d & 0xFFFFFFFF).astype(np.uint64)


def lane_of(g, order, targets):
    """The batch lane each caller target occupies when the graph has
    coordinates (cpd_gpu.cpp upload_targets: lanes sorted by (Hilbert key,
    column)).  lane_of(...)[i] = lane of targets[i]."""
    t = np.asarray(targets, np.int64)
    keys = hilbert_keys(g.x, g.y)[t]
    cols = np.asarray(order, np.uint64)[t]
    idx = np.lexsort((cols, keys))  # by key, then column
    lane = np.empty(len(t), np.int64)
    lane[idx] = np.arange(len(t))
    return lane
