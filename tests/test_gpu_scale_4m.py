"""GPU parity at BASELINE.json configs[4]: the synthetic 4M-node road graph
(2000 x 2000 lattice, seed 4), 256k targets sampled without replacement
(seed 5), partition div 8, worker 0's share (~32k rows) — one build batch at
the default width for 4M nodes (5120 rows: what ~3/4 of HBM holds), so the
narrow/wide row switching and the batch sizing run at scale.

  - 32 rows spread over the batch: bit-exact against the oracle;
  - every row of the batch well formed (sampled lanes);
  - the batch streamed into a dense index and walked (queries: s uniform over
    the graph, t uniform over the batch, SURVEY.md §8d seed 6): every walk
    finishes and free-flow cost == Dijkstra for every query of 8 targets;
  - the worker's whole ~32.7k-row index and its share of the 10M-query batch,
    as the bench serves them (test_4m_worker_index_serves_its_queries).
"""
import gc

import numpy as np
import pytest

import cpd
import oracle
from scale_common import check_row_format, owned, plan_for, sample_targets, spread

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def w4m():
    g = cpd.synth_road_graph(2000, 2000, seed=4)
    plan = plan_for(g, "synth2000-s4")
    dev = cpd.Graph(plan, device=0)  # batch from free HBM
    sample = sample_targets(g.n, 262144, seed=5)
    mine = owned(sample, 8, "div", 8, 0, g.n)
    yield g, plan, dev, mine
    del dev, plan
    gc.collect()


def test_4m_batch_bit_exact_and_walks(w4m):
    g, plan, dev, mine = w4m
    B = dev.batch
    assert 4096 <= B <= 8192, B  # 5120 on an idle MI355X
    assert len(mine) > 30000
    targets = mine[:B]
    rows = dev.build_rows(targets)
    nrows, total = rows.count()
    assert nrows == B
    for i in np.unique(np.concatenate([[0, B - 1], np.arange(0, B, 331)])):
        off, runs = rows.export_range(int(i), 1)
        check_row_format(off, runs, g.n)
    lanes = spread(np.arange(B), 32)
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets[lanes])
    for k, i in enumerate(lanes):
        off, runs = rows.export_range(int(i), 1)
        np.testing.assert_array_equal(runs, ref_runs[int(ref_off[k]):int(ref_off[k + 1])],
                                      err_msg=f"row {i} (target {targets[i]})")
    ix = cpd.Index.streamed(dev, targets, total, mode="dense")
    ix.append_rows(rows)
    del rows
    gc.collect()
    rng = np.random.default_rng(6)
    probe = rng.choice(targets, 8, replace=False)
    nq = 100_000
    s = rng.integers(0, g.n, nq).astype(np.uint32)
    t = np.where(np.arange(nq) % 4 == 0, probe[rng.integers(0, 8, nq)],
                 targets[rng.integers(0, B, nq)]).astype(np.uint32)
    keep = s != t
    s, t = s[keep], t[keep]
    cost, hops, fin, st = ix.query(s, t)
    assert fin.all()
    for tt in probe:
        d = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, tt)
        sel = t == tt
        np.testing.assert_array_equal(cost[sel], d[s[sel]].astype(np.uint64))


def test_4m_worker_index_serves_its_queries(w4m):
    """configs[4] as bench.py --workload synth4m serves it: worker 0's WHOLE
    row set (~32.7k rows, built batch by batch and streamed into one dense
    index), then its share of the 10M-query batch (t uniform over the 256k
    sample, s uniform, seed 6: ~1.25M queries).  Every walk finishes; for 16
    probe targets cost == Dijkstra and cost / moves / flags are bit-exact
    against the oracle's rows."""
    g, plan, dev, mine = w4m
    B = dev.batch
    ix = cpd.Index.streamed(dev, mine, 1 << 62, mode="dense")
    rows = None
    for a in range(0, len(mine), B):
        rows = dev.build_rows(mine[a:a + B], reuse=rows)
        ix.append_rows(rows)
    del rows
    gc.collect()
    assert ix.info()["added"] == len(mine)
    qrng = np.random.default_rng(6)
    sample = sample_targets(g.n, 262144, seed=5)
    allt = sample[qrng.integers(0, 262144, 10_000_000)]
    alls = qrng.integers(0, g.n, 10_000_000).astype(np.uint32)
    sel = np.isin(allt, mine)
    s, t = alls[sel], allt[sel].astype(np.uint32)
    assert len(s) >= 200_000, len(s)
    cost, hops, fin, st = ix.query(s, t)
    assert fin.all() and st["finished"] == len(s)
    # probes: the 16 targets with the most queries
    uniq, cnt = np.unique(t, return_counts=True)
    probe = np.sort(uniq[np.argsort(-cnt, kind="stable")[:16]])
    qsel = np.isin(t, probe)
    assert qsel.sum() >= 16
    for tt in probe:
        d = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, tt)
        m = t == tt
        np.testing.assert_array_equal(cost[m], d[s[m]].astype(np.uint64))
    order = plan.order()
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, probe)
    rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, order, probe, ref_off, ref_runs,
                                     s[qsel], t[qsel])
    np.testing.assert_array_equal(cost[qsel], rc)
    np.testing.assert_array_equal(hops[qsel], rh)
    np.testing.assert_array_equal(fin[qsel], rf)
