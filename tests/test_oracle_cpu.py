"""The CPU oracle, pinned before it is trusted.

- distances against scipy.sparse.csgraph.dijkstra (independent implementation);
- hand-worked known-answer vectors for first-move sets, RLE rows, get_move and
  table-search (tests/golden/known_answers.json, derived by hand below);
- structural properties of every RLE row (run starts strictly increase from
  column 0; every column's move is one of its optimal first moves; greedy
  maximality: no run can absorb the next column).
"""
import json
import os

import numpy as np
import pytest
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import dijkstra

import cpd
import oracle
from scale_common import move_run_counts

KA = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))


def _csr(g):
    rows = np.repeat(np.arange(g.n), np.diff(g.row_ptr.astype(np.int64)))
    # scipy keeps the minimum over duplicate entries only via min-reduction; build
    # explicitly so parallel edges keep the lightest weight
    best = {}
    for a, b, w in zip(rows, g.dst, g.w):
        if a == b:
            continue
        best[(a, b)] = min(best.get((a, b), w), w)
    if not best:
        return csr_matrix((g.n, g.n))
    ab = np.array(list(best.keys()))
    w = np.array(list(best.values()), np.float64)
    # scipy treats explicit zeros as missing: nudge zero weights, compare after rounding
    return csr_matrix((np.where(w == 0, 1e-9, w), (ab[:, 0], ab[:, 1])), shape=(g.n, g.n))


@pytest.fixture(scope="module")
def graphs():
    from graphs import GRAPHS  # the same cases as the GPU suite
    return {k: f() for k, f in GRAPHS.items()}


def test_distances_match_scipy(graphs):
    rng = np.random.default_rng(0)
    for name, g in graphs.items():
        A = _csr(g).T.tocsr()
        for t in rng.choice(g.n, size=min(g.n, 12), replace=False):
            ref = dijkstra(A, indices=[t])[0]
            got = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, t).astype(np.float64)
            got[got == oracle.INF] = np.inf
            np.testing.assert_array_equal(got, np.round(ref), err_msg=f"{name} t={t}")


def _check_row(g, order, t, runs):
    fm = oracle.first_moves(g.row_ptr, g.dst, g.w, t)
    n = g.n
    starts = runs >> 4
    assert starts[0] == 0 and np.all(np.diff(starts.astype(np.int64)) > 0)
    inv = np.empty(n, np.int64)
    inv[order] = np.arange(n)
    run_of_col = np.searchsorted(starts, np.arange(n), side="right") - 1
    moves = (runs & 0xF)[run_of_col]
    f = fm[inv].astype(np.int64)
    assert np.all((f >> moves) & 1), "a column's move is not an optimal first move"
    # greedy maximality: run r's AND with the first column of run r+1 is empty
    for r in range(len(runs) - 1):
        a, b = int(starts[r]), int(starts[r + 1])
        acc = np.bitwise_and.reduce(f[a:b + 1])
        assert acc == 0


def test_rle_rows_properties(graphs):
    rng = np.random.default_rng(3)
    for name, g in graphs.items():
        order = oracle.dfs_preorder(g.row_ptr, g.dst)
        targets = rng.choice(g.n, size=min(g.n, 10), replace=False)
        off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets)
        for i, t in enumerate(targets):
            row = runs[off[i]:off[i + 1]]
            _check_row(g, order, t, row)
            # get_move == the move of the run covering each column
            for col in (0, g.n // 2, g.n - 1):
                j = np.searchsorted(row >> 4, col, side="right") - 1
                assert oracle.get_move(row, col) == (row[j] & 0xF)


def test_compact_rows_are_the_rle_rows(graphs):
    """The compact row form (DOSCPD02, cpd_rows_export_moves) is bijective
    with the greedy RLE row: consecutive runs always carry different moves
    (a run closes at c only when S & FM(c) is empty; its move lies in S, the
    next one's in FM(c)), so the runs are exactly column 0 and every column
    whose move differs from its left neighbour's."""
    rng = np.random.default_rng(4)
    for name, g in graphs.items():
        order = oracle.dfs_preorder(g.row_ptr, g.dst)
        targets = rng.choice(g.n, size=min(g.n, 40), replace=False)
        off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets)
        for i in range(len(targets)):
            row = runs[off[i]:off[i + 1]]
            assert np.all(np.diff((row & 0xF).astype(np.int64)) != 0), name
        deg = int(np.diff(g.row_ptr.astype(np.int64)).max())
        for bits in (1, 2, 4):  # the packed widths: every move < 2^bits when deg <= 2^bits
            if max(deg, 1) > (1 << bits):
                continue
            mv = oracle.moves_from_runs(off, runs, g.n, bits)
            assert mv.shape == (len(targets), (g.n * bits + 31) // 32)
            off2, runs2 = oracle.runs_from_moves(mv, g.n, bits)
            np.testing.assert_array_equal(off2, off, err_msg=f"{name} {bits}")
            np.testing.assert_array_equal(runs2, runs, err_msg=f"{name} {bits}")
            # the bulk run counter the 1M full-batch GPU test applies
            np.testing.assert_array_equal(move_run_counts(mv, g.n, bits, chunk=5),
                                          np.diff(off.astype(np.int64)), err_msg=f"{name} {bits}")


def _ka_graph(case):
    from graphs import graph_from_edges
    return graph_from_edges(case["n"], [tuple(e) for e in case["edges"]])


@pytest.mark.parametrize("case", KA["cases"], ids=lambda c: c["name"])
def test_known_answers(case):
    g = _ka_graph(case)
    order = oracle.dfs_preorder(g.row_ptr, g.dst)
    assert order.tolist() == case["order"]
    for t_s, exp in case["rows"].items():
        t = int(t_s)
        assert oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, t).tolist() == exp["dist"]
        assert oracle.first_moves(g.row_ptr, g.dst, g.w, t).tolist() == exp["fm"]
        off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, [t])
        assert runs.tolist() == exp["runs"]
    for q in case["queries"]:
        targets = sorted({int(k) for k in case["rows"]})
        off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets)
        cost, hops, fin = oracle.table_search(g.row_ptr, g.dst, g.w, order, targets, off, runs,
                                              [q["s"]], [q["t"]])
        assert [int(cost[0]), int(hops[0]), int(fin[0])] == [q["cost"], q["hops"], q["finished"]]


def test_free_flow_extraction_is_shortest(graphs):
    rng = np.random.default_rng(8)
    for name, g in graphs.items():
        order = oracle.dfs_preorder(g.row_ptr, g.dst)
        targets = rng.choice(g.n, size=min(g.n, 8), replace=False).astype(np.uint32)
        off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets)
        s = rng.integers(0, g.n, 300).astype(np.uint32)
        t = targets[rng.integers(0, len(targets), 300)]
        cost, hops, fin = oracle.table_search(g.row_ptr, g.dst, g.w, order, targets, off, runs, s, t)
        for q in range(300):
            d = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, t[q])[s[q]]
            if d == oracle.INF:
                continue
            if np.all(g.w > 0):
                assert fin[q] == 1 and cost[q] == d, (name, q)


def test_missing_row_raises():
    g = cpd.synth_road_graph(5, 5, seed=1)
    order = oracle.dfs_preorder(g.row_ptr, g.dst)
    off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, [3])
    with pytest.raises(KeyError):
        oracle.table_search(g.row_ptr, g.dst, g.w, order, [3], off, runs, [0], [4])


# ---------------------------------------------------------------------------
# CPD-heuristic search restatement (ora_cpd_search):
# warthog's cpd_search source is absent, so the oracle is pinned by the
# properties the published algorithm guarantees.

def _search_case(w=36, seed=5, frac=0.25):
    import cpd
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    g = cpd.synth_road_graph(w, w, seed=seed)
    order = oracle.dfs_preorder(g.row_ptr, g.dst)
    rng = np.random.default_rng(seed)
    T = rng.choice(g.n, 12, replace=False).astype(np.uint32)
    off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, T)
    s = rng.integers(0, g.n, 600).astype(np.uint32)
    t = T[rng.integers(0, len(T), 600)]
    wc = cpd.synth_congestion(g.w, frac, 1.0, 3.0, seed)
    src = np.repeat(np.arange(g.n), np.diff(g.row_ptr))
    us = np.unique(s)
    D = dijkstra(csr_matrix((wc.astype(float), (src, g.dst)), shape=(g.n, g.n)), indices=us)
    row = {v: i for i, v in enumerate(us)}
    opt = np.array([D[row[a], b] for a, b in zip(s, t)])
    return g, order, T, off, runs, s, t, wc, opt


def test_search_optimal_at_default_scales():
    g, order, T, off, runs, s, t, wc, opt = _search_case()
    c, pl, f, st = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t)
    assert f.all()
    np.testing.assert_array_equal(c.astype(float), opt)      # == congested Dijkstra
    tc, th, tf = oracle.table_search(g.row_ptr, g.dst, wc, order, T, off, runs, s, t)
    assert np.all(c <= tc)                                    # never worse than the CPD path
    assert np.all(st[:, 0] >= 1) and np.all(st[:, 1] >= st[:, 0] - st[:, 3])


@pytest.mark.parametrize("fs", [0.05, 0.3, 1.0])
def test_search_bounded_suboptimal(fs):
    g, order, T, off, runs, s, t, wc, opt = _search_case()
    c, _, f, st = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t,
                                    fscale=fs)
    assert f.all() and np.all(c <= (1 + fs) * opt + 1e-9)
    c0, _, _, st0 = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t)
    assert st[:, 0].sum() <= st0[:, 0].sum()


def test_search_free_flow_is_one_expansion_and_plen_is_the_walk():
    g, order, T, off, runs, s, t, wc, opt = _search_case()
    c, pl, f, st = oracle.cpd_search(g.row_ptr, g.dst, g.w, g.w, order, T, off, runs, s, t)
    tc, th, tf = oracle.table_search(g.row_ptr, g.dst, g.w, order, T, off, runs, s, t)
    np.testing.assert_array_equal(c, tc)
    np.testing.assert_array_equal(pl, th)
    assert np.all(st[:, 0] == 1)


def test_search_limits():
    g, order, T, off, runs, s, t, wc, opt = _search_case()
    c, pl, f, st = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t,
                                     itrs=3)
    assert np.all(st[:, 0] <= 3)
    assert f.all()  # the first expansion already has the CPD path as incumbent
    c0, _, f0, st0 = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t,
                                       k_moves=0)
    # k_moves = 0: only t itself yields an incumbent, so the search ends at t
    np.testing.assert_array_equal(c0.astype(float), opt)
    assert np.all(st0[:, 0] >= 1)


def test_search_virtual_time_limit():
    """The deterministic restatement of `time`: tick_ns per expansion and per
    touched edge.  A 1-ns budget allows exactly the first expansion (its
    incumbent is the CPD path: the table-search cost); budgets grow the
    search monotonically; no budget = no limit; tick 0 = not modelled."""
    g, order, T, off, runs, s, t, wc, opt = _search_case()
    tc, th, tf = oracle.table_search(g.row_ptr, g.dst, wc, order, T, off, runs, s, t)
    c1, p1, f1, st1 = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t,
                                        time_ns=1, tick_ns=1)
    assert np.all(st1[:, 0] == 1)
    np.testing.assert_array_equal(c1, tc)
    prev = st1[:, 0].sum()
    for budget in (50, 500, 5000):
        _, _, _, stb = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t,
                                         time_ns=budget, tick_ns=1)
        assert stb[:, 0].sum() >= prev
        prev = stb[:, 0].sum()
    c0, _, _, st0 = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t)
    for kw in (dict(time_ns=0, tick_ns=1), dict(time_ns=1, tick_ns=0)):
        c, _, _, st = oracle.cpd_search(g.row_ptr, g.dst, g.w, wc, order, T, off, runs, s, t, **kw)
        np.testing.assert_array_equal(c, c0)
        np.testing.assert_array_equal(st, st0)
