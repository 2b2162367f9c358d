"""GPU parity: libcpd (HIP, gfx950) against the CPU oracle, bit-exact.

Integer work, so the bar is exact equality: distances, first-move sets, RLE
row words, per-query costs/hops/finished flags.  Inputs are seeded synthetic
road graphs plus hand-built edge cases (unreachable nodes, degree-15 nodes,
self loops, parallel edges, zero weights, a single node).
"""
import os

import numpy as np
import pytest

import cpd
import oracle
from graphs import GRAPHS, graph_from_edges

pytestmark = pytest.mark.gpu


def make_graph(plan, batch, narrow):
    """Device graph with narrow (u16-offset) distance rows on or off
    (CPD_NARROW is read when the graph is created)."""
    old = os.environ.get("CPD_NARROW")
    os.environ["CPD_NARROW"] = "1" if narrow else "0"
    try:
        return cpd.Graph(plan, batch=batch)
    finally:
        if old is None:
            del os.environ["CPD_NARROW"]
        else:
            os.environ["CPD_NARROW"] = old


# (narrow rows, lane order from coordinates): the Hilbert lane order of
# cpd_graph_set_coords must give the same rows as the column order
MODES = [(True, False), (False, False), (True, True)]


@pytest.fixture(scope="module", params=[(name, narrow, xy) for name in sorted(GRAPHS)
                                        for narrow, xy in MODES],
                ids=lambda p: f"{p[0]}-{'narrow' if p[1] else 'wide'}{'-xy' if p[2] else ''}")
def setup(request):
    name, narrow, xy = request.param
    g = GRAPHS[name]()
    plan = cpd.Plan(g)
    dev = make_graph(plan, 1024, narrow)
    if xy:  # the graph's coordinates, or seeded random ones for edge-list graphs
        rng = np.random.default_rng(5)
        x = g.x if g.x is not None else rng.integers(-1000, 1000, g.n, dtype=np.int32)
        y = g.y if g.y is not None else rng.integers(-1000, 1000, g.n, dtype=np.int32)
        dev.set_coords(x, y)
    return name, g, plan, dev


def test_distances_and_first_moves(setup):
    name, g, plan, dev = setup
    rng = np.random.default_rng(1)
    targets = rng.choice(g.n, size=min(g.n, 37), replace=False).astype(np.uint32)
    dist, fm = dev.debug_rows(targets)
    for i, t in enumerate(targets):
        ref = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, t)
        np.testing.assert_array_equal(dist[:, i], ref, err_msg=f"{name} dist t={t}")
        ref_fm = oracle.first_moves(g.row_ptr, g.dst, g.w, t)
        np.testing.assert_array_equal(fm[i], ref_fm, err_msg=f"{name} fm t={t}")


def test_rows_bit_exact(setup):
    name, g, plan, dev = setup
    targets = np.arange(g.n, dtype=np.uint32)[::-1].copy()  # all rows, reversed order
    rows = dev.build_rows(targets)
    off, runs = rows.export()
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    np.testing.assert_array_equal(off, ref_off, err_msg=name)
    np.testing.assert_array_equal(runs, ref_runs, err_msg=name)


def test_compact_rows_bit_exact(setup):
    """The rows' compact form (4-bit move per column, what DOSCPD02 files and
    dense indexes hold) against the oracle's RLE rows expanded, and both index
    forms loaded from it walk like the oracle."""
    name, g, plan, dev = setup
    rng = np.random.default_rng(6)
    targets = rng.permutation(g.n)[: min(g.n, 1500)].astype(np.uint32)
    rows = dev.build_rows(targets)
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    bits = rows.move_bits()
    deg = int(np.diff(g.row_ptr.astype(np.int64)).max())
    assert bits == (1 if deg <= 2 else 2 if deg <= 4 else 4) == dev.move_bits()
    mv = rows.export_moves()
    np.testing.assert_array_equal(mv, oracle.moves_from_runs(ref_off, ref_runs, g.n, bits),
                                  err_msg=name)
    # a range, and the decoded runs of a range
    a = len(targets) // 3
    b = min(len(targets), a + 7)
    np.testing.assert_array_equal(rows.export_moves(a, b - a), mv[a:b])
    o, r = rows.export_range(a, b - a)
    np.testing.assert_array_equal(r, ref_runs[int(ref_off[a]):int(ref_off[b])])
    np.testing.assert_array_equal(o, ref_off[a:b + 1] - ref_off[a])
    s = rng.integers(0, g.n, 3000).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), 3000)]
    rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, plan.order(), targets, ref_off,
                                     ref_runs, s, t)
    mv4 = oracle.moves_from_runs(ref_off, ref_runs, g.n, 4)
    for mode in ("dense", "rle"):
        ix = cpd.Index.streamed(dev, targets, int(ref_off[-1]), mode=mode)
        half = len(targets) // 2
        ix.append_moves(mv[:half], bits)
        ix.append_moves(mv4[half:], 4)  # any width holding the moves is accepted
        assert ix.mode == mode
        cost, hops, fin, _ = ix.query(s, t)
        np.testing.assert_array_equal(cost, rc, err_msg=f"{name} {mode}")
        np.testing.assert_array_equal(hops, rh, err_msg=f"{name} {mode}")
        np.testing.assert_array_equal(fin, rf, err_msg=f"{name} {mode}")
        if mode == "rle":
            assert ix.info()["runs_resident"] == int(ref_off[-1])


@pytest.mark.parametrize("mode", ["rle", "dense", "auto"])
def test_queries_free_flow_and_congested(setup, mode):
    name, g, plan, dev = setup
    rng = np.random.default_rng(2)
    targets = rng.choice(g.n, size=min(g.n, 50), replace=False).astype(np.uint32)
    rows = dev.build_rows(targets)
    off, runs = rows.export()
    ix = cpd.Index(dev, rows=rows)
    ix.set_mode(mode)
    assert ix.mode == (mode if mode != "auto" else ix.mode)
    nq = 4000
    s = rng.integers(0, g.n, nq).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), nq)]
    cost, hops, fin, st = ix.query(s, t)
    rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, plan.order(), targets, off, runs, s, t)
    np.testing.assert_array_equal(cost, rc)
    np.testing.assert_array_equal(hops, rh)
    np.testing.assert_array_equal(fin, rf)
    assert st["hops"] == int(rh.sum()) and st["finished"] == int(rf.sum())
    assert st["cost"] == int(rc.sum())
    # free-flow cost of a finished walk is the shortest distance
    for q in range(0, nq, 97):
        d = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, t[q])[s[q]]
        if d != oracle.INF:
            assert fin[q] == 1 and cost[q] == d
    # congested weights: same walk, other weights
    wc = cpd.synth_congestion(g.w, frac=0.3, lo=1.0, hi=3.0, seed=3)
    ix.set_weights(wc)
    cost2, hops2, fin2, _ = ix.query(s, t)
    rc2, rh2, rf2 = oracle.table_search(g.row_ptr, g.dst, wc, plan.order(), targets, off, runs, s, t)
    np.testing.assert_array_equal(cost2, rc2)
    np.testing.assert_array_equal(hops2, rh2)
    ix.set_weights(None)
    cost3, _, _, _ = ix.query(s, t)
    np.testing.assert_array_equal(cost3, rc)
    # k_moves cut-off
    cost4, hops4, fin4, _ = ix.query(s, t, k_moves=3)
    rc4, rh4, rf4 = oracle.table_search(g.row_ptr, g.dst, g.w, plan.order(), targets, off, runs,
                                        s, t, k_moves=3)
    np.testing.assert_array_equal(cost4, rc4)
    np.testing.assert_array_equal(hops4, rh4)
    np.testing.assert_array_equal(fin4, rf4)


def test_index_from_host_arrays_and_norow():
    g = GRAPHS["synth"]()
    plan = cpd.Plan(g)
    dev = cpd.Graph(plan, batch=1024)
    targets = np.arange(0, g.n, 7, dtype=np.uint32)
    rows = dev.build_rows(targets)
    off, runs = rows.export()
    a = cpd.Index(dev, rows=rows)
    b = cpd.Index(dev, row_targets=targets, offsets=off, runs=runs)
    rng = np.random.default_rng(4)
    s = rng.integers(0, g.n, 1000).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), 1000)]
    a.set_mode("rle")
    b.set_mode("dense")
    ca = a.query(s, t)
    cb = b.query(s, t)
    for x, y in zip(ca[:3], cb[:3]):
        np.testing.assert_array_equal(x, y)
    with pytest.raises(cpd.CpdError) as ei:
        a.query(np.array([0], np.uint32), np.array([1], np.uint32))  # node 1: no row
    assert ei.value.code == cpd.CPD_E_NOROW
    # empty batch
    c, h, f, st = a.query(np.zeros(0, np.uint32), np.zeros(0, np.uint32))
    assert len(c) == 0 and st["queries"] == 0


def test_multi_batch_and_reuse():
    """ntargets > batch: rows are built in several sweeps and appended in order."""
    g = cpd.synth_road_graph(50, 50, seed=9)
    plan = cpd.Plan(g)
    dev = cpd.Graph(plan, batch=1024)
    rng = np.random.default_rng(6)
    targets = rng.integers(0, g.n, 2500).astype(np.uint32)  # duplicates allowed
    rows = dev.build_rows(targets)
    off, runs = rows.export()
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    np.testing.assert_array_equal(off, ref_off)
    np.testing.assert_array_equal(runs, ref_runs)
    rows2 = dev.build_rows(targets[:100], reuse=rows)
    off2, runs2 = rows2.export()
    np.testing.assert_array_equal(off2, ref_off[:101])
    np.testing.assert_array_equal(runs2, ref_runs[: int(ref_off[100])])


@pytest.mark.parametrize("width,batch", [(60, 4096), (90, 8192), (200, 4096)])
def test_multi_slab_batches(width, batch):
    """Several 1024-target slabs per batch (slab masks, split narrow levels),
    targets in shuffled order (the batch is sorted by column internally)."""
    g = cpd.synth_road_graph(width, width, seed=width)
    plan = cpd.Plan(g)
    dev = cpd.Graph(plan, batch=batch)
    rng = np.random.default_rng(width)
    targets = rng.permutation(g.n).astype(np.uint32)[: min(g.n, batch + 1500)]
    rows = dev.build_rows(targets)
    off, runs = rows.export()
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    np.testing.assert_array_equal(off, ref_off)
    np.testing.assert_array_equal(runs, ref_runs)
    nd = min(len(targets), batch)
    dist, _ = dev.debug_rows(targets[:nd], want_fm=False)
    for i in rng.choice(nd, 5, replace=False):
        np.testing.assert_array_equal(
            dist[:, i], oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, targets[i]))


def test_next_batch_hint_and_early_up_sweep():
    """cpd_graph_hint_next: the next call's first batch starts its up-sweep
    during the current call.  A matching next call uses it, a different one
    discards it, a debug build in between drops it — rows bit-exact in every
    case; within one call, batch k + 1's up-sweep runs beside batch k's first
    moves (several batches per call, with and without coordinates)."""
    g = cpd.synth_road_graph(70, 70, seed=12)
    plan = cpd.Plan(g)
    order = plan.order()
    rng = np.random.default_rng(12)
    perm = rng.permutation(g.n).astype(np.uint32)
    A, Bt, Ct = perm[:1024], perm[1024:2048], perm[2048:2900]
    for xy in (False, True):
        dev = cpd.Graph(plan, batch=1024)
        if xy:
            dev.set_coords(g.x, g.y)

        def check(rows, tg):
            off, runs = rows.export()
            ro, rr = oracle.build_rows(g.row_ptr, g.dst, g.w, order, tg)
            np.testing.assert_array_equal(off, ro)
            np.testing.assert_array_equal(runs, rr)

        dev.hint_next(Bt)
        check(dev.build_rows(A), A)
        check(dev.build_rows(Bt), Bt)      # uses the early up-sweep
        dev.hint_next(Bt)
        check(dev.build_rows(A), A)
        check(dev.build_rows(Ct), Ct)      # hint mismatch: discarded
        dev.hint_next(A)
        check(dev.build_rows(Ct), Ct)
        dev.debug_rows(Bt[:100], want_fm=False)  # drops the pending early up-sweep
        check(dev.build_rows(A), A)
        check(dev.build_rows(perm[:3500]), perm[:3500])  # 4 batches in one call
        dev.hint_next(perm[:10])                  # a partial first batch
        check(dev.build_rows(Bt), Bt)
        check(dev.build_rows(perm[:10]), perm[:10])


def test_narrow_overflow_rows_kept_wide():
    """Edge weights x700: a wave's 256 distances spread past 0xFFFF, so the
    narrow rows cannot hold them; those group rows are kept 32-bit (base =
    wide marker) and every output stays exact.  The first full batch finds
    most group rows wide and switches narrow rows off for the second."""
    g0 = cpd.synth_road_graph(40, 40, seed=12)
    g = cpd.RoadGraph(g0.row_ptr, g0.dst, (g0.w * 700).astype(np.uint32), g0.x, g0.y)
    plan = cpd.Plan(g)
    dev = make_graph(plan, 1024, True)
    rng = np.random.default_rng(12)
    targets = rng.permutation(g.n).astype(np.uint32)[:1500]
    rows = dev.build_rows(targets)
    off, runs = rows.export()
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    np.testing.assert_array_equal(off, ref_off)
    np.testing.assert_array_equal(runs, ref_runs)
    dev2 = make_graph(plan, 1024, True)
    dist, fm = dev2.debug_rows(targets[:300])
    for i in range(0, 300, 37):
        np.testing.assert_array_equal(
            dist[:, i], oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, targets[i]))
        np.testing.assert_array_equal(fm[i], oracle.first_moves(g.row_ptr, g.dst, g.w, targets[i]))


@pytest.mark.parametrize("scale,narrow_kept", [(1, True), (700, False)])
def test_narrow_rows_switched_off_when_mostly_wide(scale, narrow_kept):
    """The first full batches count their wide group rows; when most are
    wide, narrow rows are switched off for the graph's lifetime (later builds
    record no narrow batch in the timing counters).  Rows stay bit-exact
    before, across and after the switch."""
    g0 = cpd.synth_road_graph(70, 70, seed=13)
    g = cpd.RoadGraph(g0.row_ptr, g0.dst, (g0.w * scale).astype(np.uint32), g0.x, g0.y)
    plan = cpd.Plan(g)
    dev = make_graph(plan, 1024, True)
    dev.timing(True)
    rng = np.random.default_rng(13)
    targets = rng.permutation(g.n).astype(np.uint32)[:1500]
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    for rep in range(2):
        dev.timing_reset()
        off, runs = dev.build_rows(targets).export()
        np.testing.assert_array_equal(off, ref_off)
        np.testing.assert_array_equal(runs, ref_runs)
        if rep == 1:
            assert ("group_rows" in dev.timing_get()) == narrow_kept


def chain_graph(n, seed):
    """A bidirectional path 0-1-...-(n-1), weights 1..3: every row has a
    handful of runs, each spanning thousands of columns — far past the
    chunked RLE count's 16-column look-back guess."""
    rng = np.random.default_rng(seed)
    edges = []
    for v in range(n):
        if v > 0:
            edges.append((v, v - 1, int(rng.integers(1, 4))))
        if v + 1 < n:
            edges.append((v, v + 1, int(rng.integers(1, 4))))
    return graph_from_edges(n, edges)


@pytest.mark.parametrize("n", [5000, 20000])
def test_long_runs_chunk_seams(n):
    """Rows whose runs span whole chunks of the chunked RLE count: at 5000
    nodes rle_fix rescans long stretches of each row; at 20000 a row passes
    its rescan budget and the batch is re-counted by rle_scan<false> — the
    rows are bit-exact against the oracle either way."""
    g = chain_graph(n, seed=n)
    plan = cpd.Plan(g)
    dev = cpd.Graph(plan, batch=1024)
    rng = np.random.default_rng(3)
    targets = rng.choice(g.n, size=300, replace=False).astype(np.uint32)
    rows = dev.build_rows(targets)
    off, runs = rows.export()
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    np.testing.assert_array_equal(off, ref_off)
    np.testing.assert_array_equal(runs, ref_runs)
    assert int(off[-1]) < 8 * len(targets)  # a handful of runs per row


def test_narrow_pool_overflow_rebuilds_exact():
    """Narrow rows keep the wide 256-target group rows (spread >= 0xFFFF) in a
    pool of an eighth of a full batch's group rows (at least every group row
    of one 1024-target slab).  A batch whose wide rows outgrow it is built
    again in pieces the pool holds.  Weights scaled here so that about half of
    a 4-slab batch's group rows are wide (the pool holds a quarter): the rows
    stay bit-exact, the timing counters show the rebuild, and narrow rows are
    kept (a partial batch never runs the probe that switches them off)."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    g0 = cpd.synth_road_graph(60, 60, seed=21)
    plan0 = cpd.Plan(g0)
    order = plan0.order()
    n = g0.n
    targets = np.random.default_rng(21).permutation(n).astype(np.uint32)  # k = n = 3600: 4 slabs
    B = 8192
    # lanes as the build orders them without coordinates: by column, the
    # active slabs' tail padded with the first lane's target
    lanes = targets[np.argsort(order[targets], kind="stable")]
    lanes = np.concatenate([lanes, np.full(4096 - n, lanes[0], np.uint32)])
    rows = np.repeat(np.arange(n), np.diff(g0.row_ptr))
    rev = csr_matrix((g0.w.astype(np.float64), (g0.dst, rows)), shape=(n, n))
    d = dijkstra(rev, indices=lanes)            # d[lane, node] = dist(node -> target)
    d[np.isinf(d)] = np.nan
    grp = d.reshape(16, 256, n)
    spread = np.nanmax(grp, axis=1) - np.nanmin(grp, axis=1)  # [group, column]
    scale = int(np.ceil(65535.0 / np.nanmedian(spread)))
    assert 2 <= scale <= 5000, scale
    g = cpd.RoadGraph(g0.row_ptr, g0.dst, (g0.w.astype(np.int64) * scale).astype(np.uint32),
                      g0.x, g0.y)
    plan = cpd.Plan(g)
    dev = make_graph(plan, B, True)
    dev.timing(True)
    off, runs = dev.build_rows(targets).export()
    kt = dev.timing_get()
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    np.testing.assert_array_equal(off, ref_off)
    np.testing.assert_array_equal(runs, ref_runs)
    assert kt.get("pool_rebuilds", {}).get("launches", 0) >= 1, kt
    assert "group_rows" in kt  # narrow rows still on
