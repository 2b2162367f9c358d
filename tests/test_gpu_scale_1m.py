"""GPU parity at BASELINE.json configs[3]: the synthetic 1M-node / 2.5M-edge
road graph (1000 x 1000 lattice, seed 1), partition div 8, worker 0's targets
at the batch the bench times (auto: what free HBM holds, 21504 rows on an
idle MI355X) — the bench's own workload and shape.

  - 128 rows spread over the worker's targets: bit-exact against the oracle;
  - the bench's first full batch (worker 0's first B targets, Hilbert lane
    order): every row well formed, and in EVERY 1024-lane slab the rows at
    its first, last and one interior lane bit-exact against the oracle; the
    whole batch in its compact form (what DOSCPD02 files hold): the sampled
    rows bit-exact against the oracle's runs expanded, and every row's move
    changes == its run count; then those compact rows streamed into a dense
    index (the fifo_auto load) and walked: free-flow cost == Dijkstra
    distance for every query of 16 targets;
  - congested (.diff stand-in, SURVEY.md §8d: 10% of edges x U[1, 3], seed 3)
    and free-flow queries over the oracle's 128 rows, dense and RLE: cost,
    moves and finished flags bit-exact.
"""
import gc

import numpy as np
import pytest

import cpd
import oracle
from scale_common import check_row_format, lane_of, move_run_counts, owned, plan_for, spread

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def w1m():
    g = cpd.synth_road_graph(1000, 1000, seed=1)
    plan = plan_for(g, "synth1000-s1")
    dev = cpd.Graph(plan, device=0)  # auto batch from free HBM, as bench.py runs
    dev.set_coords(g.x, g.y)  # Hilbert lane order, as the bench and make_cpd_auto run
    mine = owned(np.arange(g.n), 8, "div", 8, 0, g.n)
    yield g, plan, dev, mine
    del dev, plan
    gc.collect()


@pytest.fixture(scope="module")
def rows128(w1m):
    g, plan, dev, mine = w1m
    targets = spread(mine, 128)
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    return targets, ref_off, ref_runs


def test_1m_rows_bit_exact(w1m, rows128):
    g, plan, dev, mine = w1m
    targets, ref_off, ref_runs = rows128
    off, runs = dev.build_rows(targets).export()
    np.testing.assert_array_equal(off, ref_off)
    np.testing.assert_array_equal(runs, ref_runs)


def test_1m_full_batch(w1m):
    g, plan, dev, mine = w1m
    B = dev.batch
    print(f"auto batch at 1M nodes: {B} rows ({B // 1024} slabs)")
    assert B % 1024 == 0 and B >= 20480, B  # 21504 on an idle MI355X
    targets = mine[:B]  # bench.py batch_of(owned, B, 0)
    rows = dev.build_rows(targets)
    nrows, total = rows.count()
    assert nrows == B
    for i in np.unique(np.concatenate([[0, 1, B - 2, B - 1], np.arange(0, B, 997)])):
        off, runs = rows.export_range(int(i), 1)
        check_row_format(off, runs, g.n)
    # rows by LANE: first, last and one rotating interior lane of every slab
    lane = lane_of(g, plan.order(), targets)
    np.testing.assert_array_equal(rows.lanes(), lane)  # the restated lane order holds
    row_at = np.empty(B, np.int64)
    row_at[lane] = np.arange(B)
    want = sorted({x for sl in range(B // 1024)
                   for x in (1024 * sl, 1024 * sl + 1023, 1024 * sl + (397 * sl + 211) % 1024)})
    sample = row_at[want]
    assert len(sample) >= 3 * (B // 1024) - 2
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets[sample])
    for k, i in enumerate(sample):
        off, runs = rows.export_range(int(i), 1)
        np.testing.assert_array_equal(runs, ref_runs[int(ref_off[k]):int(ref_off[k + 1])],
                                      err_msg=f"row {i} lane {want[k]} (target {targets[i]})")
    # the whole batch in its compact form: the sampled
    # rows against the oracle's runs, every row's run count from its moves
    bits = rows.move_bits()
    assert bits == 2  # out-degree <= 4
    mv = rows.export_moves()
    assert mv.shape == (B, (g.n * bits + 31) // 32)
    np.testing.assert_array_equal(mv[sample], oracle.moves_from_runs(ref_off, ref_runs, g.n, bits))
    counts = np.diff(rows.offsets().astype(np.int64))
    np.testing.assert_array_equal(move_run_counts(mv, g.n, bits), counts)
    assert int(counts.sum()) == total
    del rows  # the compact rows streamed into a dense index, as fifo_auto loads a file
    gc.collect()
    ix = cpd.Index.streamed(dev, targets, total, mode="dense")
    for a in range(0, B, 6000):
        ix.append_moves(mv[a:a + 6000], bits)
    del mv
    gc.collect()
    rng = np.random.default_rng(7)
    probe = rng.choice(targets, 16, replace=False)
    nq = 200_000
    s = rng.integers(0, g.n, nq).astype(np.uint32)
    t = np.where(np.arange(nq) % 4 == 0, probe[rng.integers(0, 16, nq)],
                 targets[rng.integers(0, B, nq)]).astype(np.uint32)
    cost, hops, fin, st = ix.query(s, t)
    assert fin.all(), "the graph is strongly connected: every walk must reach t"
    assert st["finished"] == nq and st["hops"] == int(hops.sum())
    for tt in probe:
        d = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, tt)
        sel = t == tt
        np.testing.assert_array_equal(cost[sel], d[s[sel]].astype(np.uint64))
    # cpd-search over the same worker-sized index (21504 rows: per-row tables
    # would need 430 GB, so AUTO takes the memoised walks; forcing tables is
    # a clean CPD_E_OOM), congested weights, fscale 0.1, queries to the rows
    # the oracle built above: bit-exact
    w_cong = cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3)
    ix.set_weights(w_cong)
    sq = 1000
    ss = rng.integers(0, g.n, sq).astype(np.uint32)
    stt = targets[sample][rng.integers(0, len(sample), sq)]
    rc, rp, rf, rs = oracle.cpd_search(g.row_ptr, g.dst, g.w, w_cong, plan.order(),
                                       targets[sample], ref_off, ref_runs, ss, stt, fscale=0.1)
    gc_, gp, gf, gcnt, gst = ix.search(ss, stt, fscale=0.1)
    assert gst["overflow"] == 0 and gst["tables"] == cpd.SEARCH_FORMS["walks"]
    np.testing.assert_array_equal(gc_, rc)
    np.testing.assert_array_equal(gp, rp)
    np.testing.assert_array_equal(gf, rf)
    np.testing.assert_array_equal(gcnt.astype(np.uint64), rs)
    with pytest.raises(cpd.CpdError) as ei:
        ix.search(ss[:10], stt[:10], tables="tables")
    assert ei.value.code == cpd.CPD_E_OOM


@pytest.mark.parametrize("mode", ["dense", "rle"])
def test_1m_congested_and_free_flow_vs_oracle(w1m, rows128, mode):
    g, plan, dev, mine = w1m
    targets, ref_off, ref_runs = rows128
    # load the oracle's rows the way fifo_auto loads bucket files: in chunks
    ix = cpd.Index.streamed(dev, targets, int(ref_off[-1]), mode=mode)
    for a in range(0, 128, 40):
        b = min(128, a + 40)
        ix.append(ref_off[a:b + 1] - ref_off[a], ref_runs[int(ref_off[a]):int(ref_off[b])])
    rng = np.random.default_rng(8)
    nq = 50_000
    s = rng.integers(0, g.n, nq).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), nq)]
    w_cong = cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3)
    order = plan.order()
    for w_sel in (g.w, w_cong, g.w):
        ix.set_weights(None if w_sel is g.w else w_sel)
        rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, w_sel, order, targets, ref_off,
                                         ref_runs, s, t)
        cost, hops, fin, _ = ix.query(s, t)
        np.testing.assert_array_equal(cost, rc)
        np.testing.assert_array_equal(hops, rh)
        np.testing.assert_array_equal(fin, rf)
