"""GPU parity on the melb stand-in (BASELINE.json configs[0]-[2]; melb-both.xy
is a missing blob, BASELINE.md prescribes a synthetic 300k-node graph, seed 1,
queries seed 2, .diff = 10% of edges x U[1, 3] seed 3).  The graph follows
SURVEY.md §8(d) as written (gen_synth --style spec: 548 x 548 lattice).

configs[0] shape — partition mod 3, three workers, the reference's own flow:
  3 x make_cpd_auto started TOGETHER on one --outdir with a cold plan cache
  (make_cpds.py:58-60 launches them at once); the files must be byte-
  identical to a sequential run; then 3 resident fifo_auto and the reference
  head-node protocol (tests/driver_harness.py), free-flow and congested, each
  worker's stats line and per-query side file against the oracle.  Rows are
  built for the scenario's targets only (--targets-from): a full reverse CPD
  of this graph is ~0.55 n runs per row, ~200 GB of bucket files.
configs[1] — every one of the 300k rows built on one GPU, streamed into a
  dense index (45 GB of HBM), 1M free-flow queries: all finish, cost ==
  Dijkstra, and bit-exact against the oracle for the queries of 64 targets.
configs[2] — partition mod 8: eight workers' indexes (one GPU, in turn), the
  scenario routed by target owner, congested and free-flow, bit-exact.
"""
import gc
import os
import subprocess
import time

import numpy as np
import pytest

import cpd
import driver_harness as H
import oracle
from scale_common import check_row_format, owned, spread

pytestmark = pytest.mark.gpu
BIN = H.BIN
WIDTH = 548  # 300,304 nodes
NQ_FLOW = 3000


def _read_diff(path, g):
    w = g.w.copy()
    for line in open(path):
        p = line.split()
        if not p or p[0] != "e":
            continue
        a, b, c = map(int, p[1:4])
        for e in range(g.row_ptr[a], g.row_ptr[a + 1]):
            if g.dst[e] == b:
                w[e] = c
                break
    return w


@pytest.fixture(scope="module")
def melb(tmp_path_factory):
    d = tmp_path_factory.mktemp("melb")
    prefix = str(d / "melb-standin")
    subprocess.run([os.path.join(BIN, "gen_synth"), "--width", str(WIDTH), "--seed", "1",
                    "--style", "spec", "--out", prefix, "--queries", str(NQ_FLOW),
                    "--query-seed", "2"], check=True, capture_output=True)
    xy, diff, scen = prefix + ".xy", prefix + ".xy.diff", prefix + ".scen"
    g = cpd.synth_road_graph(WIDTH, WIDTH, seed=1, style="spec")
    assert H.get_node_num(xy) == g.n
    reqs = np.array(H.read_p2p(scen), np.uint32)
    targets = np.unique(reqs[:, 1])
    order = oracle.dfs_preorder(g.row_ptr, g.dst)
    ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets)
    wc = _read_diff(diff, g)
    assert np.any(wc != g.w)
    return dict(dir=d, xy=xy, diff=diff, scen=scen, g=g, reqs=reqs, targets=targets, order=order,
                ref_off=ref_off, ref_runs=ref_runs, wc=wc)


def _oracle_walk(m, w_sel, s, t, targets=None, off=None, runs=None):
    g = m["g"]
    return oracle.table_search(g.row_ptr, g.dst, w_sel, m["order"],
                               m["targets"] if targets is None else targets,
                               m["ref_off"] if off is None else off,
                               m["ref_runs"] if runs is None else runs, s, t)


def _make_cpds(m, outdir, concurrent):
    W = 3
    cmd = lambda wid: [os.path.join(BIN, "make_cpd_auto"), "--input", m["xy"], "--partmethod",
                       "mod", "--partkey", "3", "--workerid", str(wid), "--maxworker", str(W),
                       "--outdir", outdir, "--device", "0", "--targets-from", m["scen"]]
    if concurrent:
        procs = [subprocess.Popen(cmd(w), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                  text=True) for w in range(W)]
        outs = [p.communicate(timeout=600) for p in procs]
        codes = [p.returncode for p in procs]
    else:
        outs, codes = [], []
        for w in range(W):
            p = subprocess.run(cmd(w), capture_output=True, text=True, timeout=600)
            outs.append((p.stdout, p.stderr))
            codes.append(p.returncode)
    for c, (o, e) in zip(codes, outs):
        assert c == 0, e
        assert "rows/s" in o
    return [o for o, _ in outs]



def test_melb_mod3_concurrent_build_and_driver_flow(melb):
    m = melb
    a, b = str(m["dir"] / "index-concurrent"), str(m["dir"] / "index-sequential")
    outs = _make_cpds(m, a, concurrent=True)
    assert sum("built and cached" in o for o in outs) == 1, outs
    assert sum("loaded plan" in o for o in outs) == 2, outs
    _make_cpds(m, b, concurrent=False)
    files = sorted(f for f in os.listdir(a) if f.endswith(".cpd"))
    assert files == sorted(f for f in os.listdir(b) if f.endswith(".cpd")) and len(files) == 3
    assert not [f for f in os.listdir(a) if ".tmp" in f]
    files = sorted(f for f in os.listdir(a) if ".cpd" in f)  # the buckets' part files too
    assert files == sorted(f for f in os.listdir(b) if ".cpd" in f)
    for f in files:
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f
    W = 3
    procs = []
    try:
        for wid in range(W):
            fifo = f"/tmp/worker{wid}.fifo"
            if os.path.exists(fifo):
                os.remove(fifo)
            procs.append(subprocess.Popen(
                [os.path.join(BIN, "fifo_auto"), "--input", m["xy"], m["diff"], "--partmethod",
                 "mod", "--partkey", "3", "--workerid", str(wid), "--maxworker", str(W),
                 "--outdir", a, "--alg", "table-search", "--device", "0"],
                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        for pr in procs:
            H.wait_ready(pr, timeout=300)
        nfs = str(m["dir"] / "nfs")
        os.makedirs(nfs, exist_ok=True)
        conf = {"workers": ["localhost"] * W, "nfs": nfs, "partmethod": "mod", "partkey": 3,
                "xy_file": m["xy"], "scenfile": m["scen"], "diffs": ["-", m["diff"]]}
        parts, stats = H.run(conf, dict(H.DEFAULT_CONFIG, debug=True))
        assert len(parts) == W and sum(len(p) for p in parts) == NQ_FLOW
        for x, w_sel in enumerate([m["g"].w, m["wc"]]):
            for wid, (part, row) in enumerate(zip(parts, stats[x])):
                s = np.array([q[0] for q in part], np.uint32)
                t = np.array([q[1] for q in part], np.uint32)
                rc, rh, rf = _oracle_walk(m, w_sel, s, t)
                assert int(row[0]) == int(rh.sum()) == int(row[5])  # n_expanded, plen
                assert int(row[6]) == int(rf.sum()) == len(part)
                if x == 1:
                    res = np.loadtxt(os.path.join(nfs, f"query.localhost{wid}.res"),
                                     dtype=np.uint64, ndmin=2)
                    np.testing.assert_array_equal(res[:, 2], rc)
                    np.testing.assert_array_equal(res[:, 3], rh)
    finally:
        for wid, pr in enumerate(procs):
            if pr.poll() is None:
                try:
                    with open(f"/tmp/worker{wid}.fifo", "w") as f:
                        f.write("quit\n")
                    pr.wait(timeout=30)
                except Exception:
                    pr.kill()
            fifo = f"/tmp/worker{wid}.fifo"
            if os.path.exists(fifo):
                os.remove(fifo)


def test_melb_full_build_free_flow(melb):
    m = melb
    g = m["g"]
    plan = cpd.Plan(g)
    dev = cpd.Graph(plan, device=0)
    B = dev.batch
    everything = np.arange(g.n, dtype=np.uint32)
    probe = spread(everything, 64)
    p_off, p_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, m["order"], probe)
    ix = cpd.Index.streamed(dev, everything, 1 << 40, mode="dense")
    rows = None
    checked = 0
    for a in range(0, g.n, B):
        tg = everything[a:a + B]
        rows = dev.build_rows(tg, reuse=rows)
        mine = np.nonzero((probe >= a) & (probe < a + len(tg)))[0]
        for k in mine:
            off, runs = rows.export_range(int(probe[k] - a), 1)
            check_row_format(off, runs, g.n)
            np.testing.assert_array_equal(runs, p_runs[int(p_off[k]):int(p_off[k + 1])])
            checked += 1
        ix.append_rows(rows)
    assert checked == len(probe)
    del rows
    gc.collect()
    assert ix.info()["added"] == g.n
    # the full.scen stand-in: 1M random queries (gen_synth's seed-2 stream)
    prefix = str(m["dir"] / "q1m")
    subprocess.run([os.path.join(BIN, "gen_synth"), "--width", str(WIDTH), "--seed", "1",
                    "--style", "spec", "--out", prefix, "--queries", "1000000",
                    "--query-seed", "2"], check=True, capture_output=True)
    q = np.array(H.read_p2p(prefix + ".scen"), np.uint32)
    np.testing.assert_array_equal(q[:NQ_FLOW], m["reqs"])  # same stream as the driver flow
    s, t = q[:, 0].copy(), q[:, 1].copy()
    cost, hops, fin, st = ix.query(s, t)
    assert fin.all() and st["queries"] == len(q)
    for tt in probe[::8]:
        d = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, tt)
        sel = t == tt
        np.testing.assert_array_equal(cost[sel], d[s[sel]].astype(np.uint64))
    sel = np.isin(t, probe)
    assert sel.sum() > 100
    rc, rh, rf = _oracle_walk(m, g.w, s[sel], t[sel], probe, p_off, p_runs)
    np.testing.assert_array_equal(cost[sel], rc)
    np.testing.assert_array_equal(hops[sel], rh)
    del ix, dev
    gc.collect()


def test_melb_mod8_congested(melb):
    m = melb
    g = m["g"]
    plan = cpd.Plan(g, hierarchy=True)
    dev = cpd.Graph(plan, device=0, batch=1024)
    s_all, t_all = m["reqs"][:, 0], m["reqs"][:, 1]
    served = 0
    for wid in range(8):
        mine = owned(m["targets"], 8, "mod", 8, wid, g.n)
        if not len(mine):
            continue
        rows = dev.build_rows(mine)
        ix = cpd.Index.streamed(dev, mine, rows.count()[1], mode="auto")
        ix.append_rows(rows)
        sel = np.isin(t_all, mine)
        s, t = s_all[sel], t_all[sel]
        for w_sel in (m["wc"], g.w):
            ix.set_weights(None if w_sel is g.w else w_sel)
            cost, hops, fin, _ = ix.query(s, t)
            rc, rh, rf = _oracle_walk(m, w_sel, s, t)
            np.testing.assert_array_equal(cost, rc)
            np.testing.assert_array_equal(hops, rh)
            np.testing.assert_array_equal(fin, rf)
        served += len(s)
        del ix, rows
    assert served == NQ_FLOW
