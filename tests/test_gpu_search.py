"""GPU: the CPD-heuristic search (cpd_query_search; SURVEY.md §8f item 4,
args.py:29-57) against the oracle's restatement (oracle/cpd_oracle.c
ora_cpd_search) — per query cost, plen, finished and the five search
counters, bit-exact — over hscale / fscale / k_moves / itrs, free-flow and
congested weights, dense and RLE-loaded indexes, plus the properties that
pin the restatement: optimal (== congested Dijkstra) at hscale 1, fscale 0;
within (1 + fscale) of it otherwise."""
import numpy as np
import pytest
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import dijkstra

import cpd
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    g = cpd.synth_road_graph(64, 48, seed=31)
    plan = cpd.Plan(g)
    dev = cpd.Graph(plan, batch=1024)
    rng = np.random.default_rng(31)
    targets = rng.choice(g.n, size=60, replace=False).astype(np.uint32)
    off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, plan.order(), targets)
    nq = 3000
    s = rng.integers(0, g.n, nq).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), nq)]
    wc = cpd.synth_congestion(g.w, frac=0.2, lo=1.0, hi=3.0, seed=4)
    return g, plan, dev, targets, off, runs, s, t, wc


def _oracle(env_, w_sel, **kw):
    g, plan, dev, targets, off, runs, s, t, wc = env_
    return oracle.cpd_search(g.row_ptr, g.dst, g.w, w_sel, plan.order(), targets, off, runs, s,
                             t, **kw)


def _index(env_, mode):
    g, plan, dev, targets, off, runs = env_[:6]
    ix = cpd.Index.streamed(dev, targets, int(off[-1]), mode=mode)
    ix.append(off, runs)
    return ix


@pytest.mark.parametrize("form", ["tables", "walks"])
@pytest.mark.parametrize("mode", ["dense", "rle"])
@pytest.mark.parametrize("opts", [dict(), dict(hscale=1.5), dict(fscale=0.25),
                                  dict(hscale=0.5, fscale=0.1), dict(k_moves=40),
                                  dict(itrs=7), dict(k_moves=0, itrs=200)],
                         ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()) or "default")
def test_search_matches_oracle(env, mode, opts, form):
    """Both forms of the CPD path values — per-row tables and memoised walks
    — give the oracle's results and counters."""
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, mode)
    for w_sel in (wc, g.w):
        ix.set_weights(None if w_sel is g.w else w_sel)
        rc, rp, rf, rs = _oracle(env, w_sel, **opts)
        cost, plen, fin, cnt, st = ix.search(s, t, tables=form, **opts)
        assert st["overflow"] == 0 and st["tables"] == cpd.SEARCH_FORMS[form]
        np.testing.assert_array_equal(cost, rc)
        np.testing.assert_array_equal(plen, rp)
        np.testing.assert_array_equal(fin, rf)
        np.testing.assert_array_equal(cnt.astype(np.uint64), rs)
        assert st["expanded"] == int(rs[:, 0].sum()) and st["finished"] == int(rf.sum())
        assert st["plen"] == int(rp[rf == 1].sum())


def test_search_optimal_and_bounded(env):
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    src = np.repeat(np.arange(g.n), np.diff(g.row_ptr))
    D = dijkstra(csr_matrix((wc.astype(float), (src, g.dst)), shape=(g.n, g.n)),
                 indices=np.unique(s))
    row = {v: i for i, v in enumerate(np.unique(s))}
    opt = np.array([D[row[a], b] for a, b in zip(s, t)])
    cost, plen, fin, cnt, st = ix.search(s, t)
    assert fin.all()
    np.testing.assert_array_equal(cost.astype(float), opt)
    # table-search under the same weights is never better than the search
    tc, _, _, _ = ix.query(s, t)
    assert np.all(cost <= tc)
    for fs in (0.1, 0.5):
        c2, _, f2, cnt2, _ = ix.search(s, t, fscale=fs)
        assert f2.all() and np.all(c2 <= (1 + fs) * opt + 1e-9)
        assert cnt2[:, 0].sum() <= cnt[:, 0].sum()
    # free-flow weights: the CPD path is optimal, the search stops at once
    ix.set_weights(None)
    c3, _, _, cnt3, _ = ix.search(s, t)
    np.testing.assert_array_equal(c3, ix.query(s, t)[0])
    assert np.all(cnt3[:, 0] == 1)


def test_search_overflow_is_counted_tables(env):
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    rc, rp, rf, rs = _oracle(env, wc)
    need = rs[:, 1].max()  # most nodes any query inserts
    cap = 64
    assert need > cap
    cost, plen, fin, cnt, st = ix.search(s, t, capacity=cap, tables="tables")
    assert st["overflow"] >= 1
    # pushes = inserted + updated bound a search's nodes and heap entries; a
    # search stops before a pop whose expansion (<= 4 pushes on this graph)
    # might not fit: those with room for it are exact, those above stop
    small = rs[:, 1] + rs[:, 3] + 4 <= cap
    assert small.sum() > 100
    np.testing.assert_array_equal(cost[small], rc[small])
    np.testing.assert_array_equal(cnt[small].astype(np.uint64), rs[small])
    assert (fin[rs[:, 1] > cap] == 2).all()  # stopped on the workspace, not unfinished
    assert int((fin == 2).sum()) == st["overflow"]
    # the sums hold every query's counters, overflowed ones included
    assert st["expanded"] == int(cnt[:, 0].astype(np.uint64).sum())
    assert st["inserted"] == int(cnt[:, 1].astype(np.uint64).sum())


def test_search_overflow_is_counted_walks(env):
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    rc, rp, rf, rs = _oracle(env, wc, columns=True)
    cap = 256
    assert rs[:, 5].max() > cap  # some query's walks and search meet more columns
    cost, plen, fin, cnt, st = ix.search(s, t, capacity=cap, tables="walks")
    assert st["overflow"] >= 1
    # a search's workspace holds every column its walks and search met (the
    # oracle's 6th stat) and its heap at most inserted + updated pushes (+ the
    # room one expansion needs): searches within it are exact, the others stop
    small = (rs[:, 5] <= cap) & (rs[:, 1] + rs[:, 3] + 4 <= cap)
    assert small.sum() > 100
    np.testing.assert_array_equal(cost[small], rc[small])
    np.testing.assert_array_equal(cnt[small].astype(np.uint64), rs[small, :5])
    assert (fin[rs[:, 5] > cap] == 2).all()
    assert int((fin == 2).sum()) == st["overflow"]
    assert st["expanded"] == int(cnt[:, 0].astype(np.uint64).sum())
    assert st["inserted"] == int(cnt[:, 1].astype(np.uint64).sum())


@pytest.mark.parametrize("form", ["tables", "walks"])
def test_search_capacity_escalation(env, form):
    """Searches that overflow a small workspace stop before the pop, spill
    their state and resume at 4x the capacity until none does: every result
    and counter (and the sums) the oracle's, nothing thrown away."""
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    rc, rp, rf, rs = _oracle(env, wc)
    _, _, fin1, _, st1 = ix.search(s, t, capacity=64, tables=form)
    assert st1["overflow"] > 0 and st1["reruns"] == 0 and st1["passes"] == 1
    cost, plen, fin, cnt, st = ix.search(s, t, capacity=64, capacity_max=4096, tables=form)
    assert st["overflow"] == 0 and st["reruns"] >= st1["overflow"] and st["resumed"] > 0
    # no expansion is thrown away (with walks, a search whose first walk
    # outgrows the workspace starts over before expanding anything)
    assert st["wasted_expanded"] == 0 and st["passes"] >= 2
    if form == "tables":
        assert st["restarted"] == 0 and st["resumed"] >= st1["overflow"]
    np.testing.assert_array_equal(cost, rc)
    np.testing.assert_array_equal(plen, rp)
    np.testing.assert_array_equal(fin, rf)
    np.testing.assert_array_equal(cnt.astype(np.uint64), rs)
    assert st["expanded"] == int(rs[:, 0].sum()) and st["inserted"] == int(rs[:, 1].sum())
    assert st["finished"] == int(rf.sum()) and st["plen"] == int(rp[rf == 1].sum())
    # a capacity_max that still leaves some overflowing: those report 2
    _, _, fin3, cnt3, st3 = ix.search(s, t, capacity=64, capacity_max=256, tables=form)
    assert int((fin3 == 2).sum()) == st3["overflow"] <= st1["overflow"]
    assert not (fin3 == 3).any()
    assert st3["expanded"] == int(cnt3[:, 0].astype(np.uint64).sum())


@pytest.mark.parametrize("form", ["tables", "walks"])
def test_search_spill_pool_full_restarts(env, form, monkeypatch):
    """A spill pool too small for every record: the searches whose records
    do not fit restart from scratch at the next capacity (their first pass
    counted as wasted), the others resume — the same results either way."""
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    rc, rp, rf, rs = _oracle(env, wc)
    monkeypatch.setenv("CPD_SEARCH_POOL_WORDS", "60000")
    cost, plen, fin, cnt, st = ix.search(s, t, capacity=64, capacity_max=4096, tables=form)
    assert st["restarted"] > 0 and st["resumed"] > 0 and st["wasted_expanded"] > 0
    assert st["overflow"] == 0
    np.testing.assert_array_equal(cost, rc)
    np.testing.assert_array_equal(plen, rp)
    np.testing.assert_array_equal(fin, rf)
    np.testing.assert_array_equal(cnt.astype(np.uint64), rs)
    assert st["expanded"] == int(rs[:, 0].sum())


def test_search_capacity_max_beyond_hbm(env):
    """capacity_max far above what fits: the passes grow only
    as far as 64 lanes fit in the workspace share, nothing is thrown, and
    what still overflows reports finished = 2; the rest is exact."""
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    rc, rp, rf, rs = _oracle(env, wc, columns=True)
    cost, plen, fin, cnt, st = ix.search(s, t, capacity=64, capacity_max=1 << 24, tables="walks",
                                         workspace_frac=2e-5)
    assert st["capacity_last"] < (1 << 24)
    assert int((fin == 2).sum()) == st["overflow"]
    assert st["expanded"] == int(cnt[:, 0].astype(np.uint64).sum())
    assert st["touched"] == int(cnt[:, 2].astype(np.uint64).sum())
    ok = fin != 2
    assert ok.sum() > 100
    np.testing.assert_array_equal(cost[ok], rc[ok])
    np.testing.assert_array_equal(cnt[ok].astype(np.uint64), rs[ok, :5])
    np.testing.assert_array_equal(fin[ok], rf[ok])


def test_search_auto_policy(env):
    """capacity 0: the library's workspace policy (fifo_auto's) — a first
    pass at <= 2^15 columns, escalation to 4 n, the whole request exact."""
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    for fs in (0.0, 0.1):
        rc, rp, rf, rs = _oracle(env, wc, fscale=fs)
        cost, plen, fin, cnt, st = ix.search(s, t, fscale=fs, tables="walks")
        assert st["overflow"] == 0 and 1024 <= st["capacity"] <= (1 << 15)
        np.testing.assert_array_equal(cost, rc)
        np.testing.assert_array_equal(fin, rf)
        np.testing.assert_array_equal(cnt.astype(np.uint64), rs)


@pytest.mark.parametrize("form", ["tables", "walks"])
@pytest.mark.parametrize("time_ns,tick", [(1, 1), (40, 1), (300, 3), (5000, 7), (10**12, 1)])
def test_search_time_limit_virtual_clock(env, time_ns, tick, form):
    """The time limit under the deterministic clock (tick per expansion and
    per touched edge, the oracle's restatement): bit-exact."""
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    rc, rp, rf, rs = _oracle(env, wc, time_ns=time_ns, tick_ns=tick)
    cost, plen, fin, cnt, st = ix.search(s, t, time_ns=time_ns, virtual_tick_ns=tick,
                                         tables=form)
    np.testing.assert_array_equal(cost, rc)
    np.testing.assert_array_equal(plen, rp)
    np.testing.assert_array_equal(fin, rf)
    np.testing.assert_array_equal(cnt.astype(np.uint64), rs)


@pytest.mark.parametrize("form", ["tables", "walks"])
def test_search_time_limit_wall_clock(env, form):
    """The wall-clock limit fifo_auto runs (time from the worker JSON): 1 ns
    (one 100-MHz tick) has passed by the first check — the start of a search
    reads HBM several times — so no search expands: the oracle at itrs = 0;
    a limit of 1000 s changes nothing."""
    g, plan, dev, targets, off, runs, s, t, wc = env
    ix = _index(env, "dense")
    ix.set_weights(wc)
    for time_ns, ref in ((1, _oracle(env, wc, itrs=0)), (10**12, _oracle(env, wc))):
        cost, plen, fin, cnt, st = ix.search(s, t, time_ns=time_ns, tables=form)
        np.testing.assert_array_equal(cost, ref[0])
        np.testing.assert_array_equal(plen, ref[1])
        np.testing.assert_array_equal(fin, ref[2])
        np.testing.assert_array_equal(cnt.astype(np.uint64), ref[3])
