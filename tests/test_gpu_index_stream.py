"""GPU: the streamed table-search index (cpd_index_create_empty + append) —
what fifo_auto loads a worker's buckets with (make_fifos.py:21 serves every
CPD the worker owns) — against the CPU oracle, bit-exact, plus its error
behaviour on malformed, incomplete or mismatched input."""
import os

import numpy as np
import pytest

import cpd
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    g = cpd.synth_road_graph(56, 44, seed=21)
    plan = cpd.Plan(g)
    dev = cpd.Graph(plan, batch=1024)
    rng = np.random.default_rng(21)
    targets = rng.choice(g.n, size=700, replace=False).astype(np.uint32)
    off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    nq = 6000
    s = rng.integers(0, g.n, nq).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), nq)]
    ref = oracle.table_search(g.row_ptr, g.dst, g.w, plan.order(), targets, off, runs, s, t)
    wc = cpd.synth_congestion(g.w, frac=0.3, lo=1.0, hi=3.0, seed=5)
    ref_c = oracle.table_search(g.row_ptr, g.dst, wc, plan.order(), targets, off, runs, s, t)
    return g, plan, dev, targets, off, runs, s, t, ref, wc, ref_c


def _check(ix, env_):
    g, plan, dev, targets, off, runs, s, t, ref, wc, ref_c = env_
    cost, hops, fin, st = ix.query(s, t)
    np.testing.assert_array_equal(cost, ref[0])
    np.testing.assert_array_equal(hops, ref[1])
    np.testing.assert_array_equal(fin, ref[2])
    assert st["hops"] == int(ref[1].sum()) and st["cost"] == int(ref[0].sum())
    ix.set_weights(wc)
    cost2, hops2, fin2, _ = ix.query(s, t)
    np.testing.assert_array_equal(cost2, ref_c[0])
    np.testing.assert_array_equal(hops2, ref_c[1])
    ix.set_weights(None)
    k = oracle.table_search(g.row_ptr, g.dst, g.w, plan.order(), targets, off, runs, s, t,
                            k_moves=5)
    c4, h4, f4, _ = ix.query(s, t, k_moves=5)
    np.testing.assert_array_equal(c4, k[0])
    np.testing.assert_array_equal(h4, k[1])
    np.testing.assert_array_equal(f4, k[2])


def _chunks(n, rng):
    cuts = np.sort(rng.choice(np.arange(1, n), size=6, replace=False))
    return [0] + list(cuts) + [n]


@pytest.mark.parametrize("mode", ["dense", "rle", "auto"])
def test_streamed_host_chunks(env, mode):
    g, plan, dev, targets, off, runs = env[:6]
    ix = cpd.Index.streamed(dev, targets, int(off[-1]), mode=mode)
    rng = np.random.default_rng(3)
    cuts = _chunks(len(targets), rng)
    for a, b in zip(cuts[:-1], cuts[1:]):
        ix.append(off[a:b + 1] - off[a], runs[int(off[a]):int(off[b])])
    info = ix.info()
    assert info["added"] == len(targets)
    if ix.mode == "dense":
        assert info["runs_resident"] == 0 and info["dense_bytes"] > 0
    else:
        assert info["runs_resident"] == int(off[-1])
    _check(ix, env)


def test_streamed_from_built_batches(env):
    """Rows built batch by batch on the GPU, expanded into the dense index as
    they come (the bench's 4M query leg), then walked."""
    g, plan, dev, targets = env[:4]
    ix = cpd.Index.streamed(dev, targets, 1 << 40, mode="dense")
    rows = None
    for a in range(0, len(targets), 256):
        rows = dev.build_rows(targets[a:a + 256], reuse=rows)
        ix.append_rows(rows)
    _check(ix, env)
    with pytest.raises(cpd.CpdError):
        ix.set_mode("rle")  # the runs were never kept


def test_incomplete_and_overfull(env):
    g, plan, dev, targets, off, runs, s, t = env[:8]
    ix = cpd.Index.streamed(dev, targets, int(off[-1]), mode="rle")
    ix.append(off[:11] - off[0], runs[: int(off[10])])
    with pytest.raises(cpd.CpdError) as ei:
        ix.query(s, t)
    assert ei.value.code == cpd.CPD_E_ARG and "incomplete" in str(ei.value)
    ix.append(off[10:] - off[10], runs[int(off[10]):])
    with pytest.raises(cpd.CpdError):
        ix.append(off[:2] - off[0], runs[: int(off[1])])  # more rows than declared
    small = cpd.Index.streamed(dev, targets, 10, mode="rle")  # declared runs too few
    with pytest.raises(cpd.CpdError):
        small.append(off[:3] - off[0], runs[: int(off[2])])


@pytest.mark.parametrize("mode", ["dense", "rle"])
def test_malformed_rows_rejected(env, mode):
    g, plan, dev, targets, off, runs = env[:6]
    two = runs[: int(off[2])].copy()
    o2 = off[:3] - off[0]
    bad_start = two.copy()
    bad_start[0] |= 5 << 4                      # first run not at column 0
    bad_order = two.copy()
    bad_order[2] = bad_order[1]                 # columns not increasing
    bad_col = two.copy()
    bad_col[int(o2[1]) - 1] = (g.n << 4) | 1    # column >= n
    # at the kernels' 512-run chunk seams (rows here hold ~1500 runs)
    assert int(o2[1]) > 1100
    seam = two.copy()
    seam[512] = seam[511]
    seam2 = two.copy()
    seam2[1024] = seam2[1023] - (1 << 4)
    for r in (bad_start, bad_order, bad_col, seam, seam2):
        ix = cpd.Index.streamed(dev, targets[:2], int(o2[-1]), mode=mode)
        with pytest.raises(cpd.CpdError) as ei:
            ix.append(o2, r)
        assert ei.value.code == cpd.CPD_E_ARG


@pytest.mark.parametrize("mode", ["dense", "rle"])
def test_move_naming_no_edge_stops_walk(env, mode):
    """A run whose move names no out-edge of the column it is applied at ends
    that walk unfinished — exactly the oracle's break — and never reads
    another column's adjacency slots."""
    g, plan, dev, targets, off, runs = env[:6]
    deg = np.diff(g.row_ptr)
    order = plan.order()
    r = runs[: int(off[1])].copy()
    r = (r & ~np.uint32(0xF)) | np.uint32(15)   # every move = 15: no such edge
    ix = cpd.Index.streamed(dev, targets[:1], len(r), mode=mode)
    if mode == "dense" and dev.move_bits() < 4:
        # this graph's tables hold 1- or 2-bit moves: such a row is refused,
        # never truncated into a move that names a real edge
        with pytest.raises(cpd.CpdError) as ei:
            ix.append(np.array([0, len(r)], np.uint64), r)
        assert ei.value.code == cpd.CPD_E_ARG and "moves <" in str(ei.value)
        return
    ix.append(np.array([0, len(r)], np.uint64), r)
    s = np.where(deg > 0)[0][:50].astype(np.uint32)
    s = s[s != targets[0]]
    t = np.full(len(s), targets[0], np.uint32)
    rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, order, targets[:1],
                                     np.array([0, len(r)], np.uint64), r, s, t)
    c, h, f, _ = ix.query(s, t)
    np.testing.assert_array_equal(c, rc)
    np.testing.assert_array_equal(h, rh)
    np.testing.assert_array_equal(f, rf)
    assert not f.any() and not h.any()


@pytest.mark.parametrize("mode", ["dense", "rle"])
def test_crafted_row_lengths(env, mode):
    """Rows of 1, 2, 511, 512, 513, 1025 and n runs (random starts, random
    moves 0..3, some naming no edge): the dense expansion's run chunks and
    their 8-run lookahead, against the oracle's walk over the same rows."""
    g, plan, dev = env[:3]
    rng = np.random.default_rng(9)
    lens = [1, 2, 511, 512, 513, 1025, g.n]
    targets = rng.choice(g.n, size=len(lens), replace=False).astype(np.uint32)
    rows = []
    for R in lens:
        cols = np.sort(rng.choice(np.arange(1, g.n), size=R - 1, replace=False)) if R > 1 else []
        cols = np.concatenate([[0], cols]).astype(np.uint32)
        rows.append((cols << 4) | rng.integers(0, 4, R).astype(np.uint32))
    off = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.uint64)
    runs = np.concatenate(rows).astype(np.uint32)
    ix = cpd.Index.streamed(dev, targets, int(off[-1]), mode=mode)
    ix.append(off, runs)
    nq = 3000
    s = rng.integers(0, g.n, nq).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), nq)]
    rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, plan.order(), targets, off, runs, s, t)
    cost, hops, fin, _ = ix.query(s, t)
    np.testing.assert_array_equal(cost, rc)
    np.testing.assert_array_equal(hops, rh)
    np.testing.assert_array_equal(fin, rf)


@pytest.mark.parametrize("mode", ["dense", "rle"])
def test_compact_rows_wider_than_tables(env, mode):
    """4-bit compact rows into an index whose tables are narrower (the graph's
    out-degree <= 4): valid rows are repacked bit-exact; a row carrying a move
    the tables cannot hold is refused (never truncated)."""
    g, plan, dev, targets, off, runs = env[:6]
    if dev.move_bits() == 4:
        pytest.skip("this graph's tables are 4-bit")
    k = 5
    mv4 = oracle.moves_from_runs(off[:k + 1], runs, g.n, 4)
    ix = cpd.Index.streamed(dev, targets[:k], int(off[k]), mode=mode)
    ix.append_moves(mv4, 4)
    rng = np.random.default_rng(3)
    s = rng.integers(0, g.n, 2000).astype(np.uint32)
    t = targets[:k][rng.integers(0, k, 2000)]
    rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, plan.order(), targets[:k],
                                     off[:k + 1], runs[: int(off[k])], s, t)
    c, h, f, _ = ix.query(s, t)
    np.testing.assert_array_equal(c, rc)
    np.testing.assert_array_equal(h, rh)
    np.testing.assert_array_equal(f, rf)
    bad = mv4.copy()
    bad[0, 0] |= np.uint32(0xF)  # column 0 of row 0: move 15
    ix2 = cpd.Index.streamed(dev, targets[:k], int(off[k]) + 2, mode=mode)
    with pytest.raises(cpd.CpdError) as ei:
        ix2.append_moves(bad, 4)
    assert ei.value.code == cpd.CPD_E_ARG
