"""End-to-end drop-in test on the GPU: our executables driven exactly the way
the reference drivers drive warthog's (make_cpds.py:20, make_fifos.py:21,
process_query.py:35-111), with `ssh host 'bash -s'` replaced by local bash
(tests/driver_harness.py; bytes pinned by tests/golden/driver_fixtures.json).
The answers and per-query side files are checked against the CPU oracle."""
import os
import subprocess
import time

import numpy as np
import pytest

import cpd
import driver_harness as H
import oracle

pytestmark = pytest.mark.gpu
BIN = H.BIN


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



@pytest.mark.parametrize("method,key,fmt", [("mod", 3, "moves"), ("div", 5, "moves"),
                                            ("mod", 3, "rle")])
def test_drivers_end_to_end(tmp_path, method, key, fmt):
    """fmt: the bucket layout make_cpd_auto writes (DOSCPD02 move tables by
    default, DOSCPD01 run words with --format rle); fifo_auto reads either."""
    W = 3
    prefix = str(tmp_path / "g")
    subprocess.run([os.path.join(BIN, "gen_synth"), "--width", "30", "--height", "24", "--seed",
                    "2", "--out", prefix, "--queries", "3000"], check=True, capture_output=True)
    xy, diff, scen = prefix + ".xy", prefix + ".xy.diff", prefix + ".scen"
    outdir = str(tmp_path / "index")
    for wid in range(W):
        p = subprocess.run([os.path.join(BIN, "make_cpd_auto"), "--input", xy, "--partmethod", method,
                            "--partkey", str(key), "--workerid", str(wid), "--maxworker", str(W),
                            "--outdir", outdir, "--device", "0", "--format", fmt],
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr
        assert "rows/s" in p.stdout
    g = cpd.synth_road_graph(30, 24, seed=2)
    order = oracle.dfs_preorder(g.row_ptr, g.dst)
    wc = _read_diff(diff, g)
    assert np.any(wc != g.w)

    procs = []
    try:
        for wid in range(W):
            fifo = f"/tmp/worker{wid}.fifo"
            if os.path.exists(fifo):
                os.remove(fifo)
            procs.append(subprocess.Popen(
                [os.path.join(BIN, "fifo_auto"), "--input", xy, diff, "--partmethod", method,
                 "--partkey", str(key), "--workerid", str(wid), "--maxworker", str(W), "--outdir",
                 outdir, "--alg", "table-search", "--device", "0"],
                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        for pr in procs:
            H.wait_ready(pr, timeout=60)
        nfs = str(tmp_path / "nfs")
        os.makedirs(nfs)
        conf = {"workers": ["localhost"] * W, "nfs": nfs, "partmethod": method, "partkey": key,
                "xy_file": xy, "scenfile": scen, "diffs": ["-", diff]}
        config = dict(H.DEFAULT_CONFIG, debug=True)
        parts, stats = H.run(conf, config)
        assert len(stats) == 2 and all(len(s) == len(parts) for s in stats)
        for x, (dname, w_sel) in enumerate([("-", g.w), (diff, wc)]):
            for wid, (part, row) in enumerate(zip(parts, stats[x])):
                assert len(row) == 13, row                  # 10 stats + t_prepare, t_partition, size
                s = np.array([q[0] for q in part], np.uint32)
                t = np.array([q[1] for q in part], np.uint32)
                targets = np.unique(t)
                off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets)
                rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, w_sel, order, targets, off, runs,
                                                 s, t)
                assert int(row[0]) == int(rh.sum())         # n_expanded = moves
                assert int(row[5]) == int(rh.sum())         # plen
                assert int(row[6]) == int(rf.sum()) == len(part)
                assert row[-1] == len(part)
                if x == 1:  # the side file holds the last experiment (congested)
                    res = np.loadtxt(os.path.join(nfs, f"query.localhost{wid}.res"),
                                     dtype=np.uint64, ndmin=2)
                    np.testing.assert_array_equal(res[:, 0], s)
                    np.testing.assert_array_equal(res[:, 2], rc)  # per-query cost
                    np.testing.assert_array_equal(res[:, 3], rh)
    finally:
        for wid, pr in enumerate(procs):
            if pr.poll() is None:
                try:
                    with open(f"/tmp/worker{wid}.fifo", "w") as f:
                        f.write("quit\n")
                    pr.wait(timeout=20)
                except Exception:
                    pr.kill()
            fifo = f"/tmp/worker{wid}.fifo"
            if os.path.exists(fifo):
                os.remove(fifo)


def _read_bucket(path):
    """The bucket layout of csrc/cpd_io.cpp (write_bucket / BucketFile)."""
    raw = open(path, "rb").read()
    assert raw[:8] == b"DOSCPD01"
    n, nrows, bid, method, key, maxworker = np.frombuffer(raw, np.uint32, 6, 8)
    total = int(np.frombuffer(raw, np.uint64, 1, 32)[0])
    p = 48
    targets = np.frombuffer(raw, np.uint32, nrows, p)
    p += 4 * int(nrows)
    off = np.frombuffer(raw, np.uint64, nrows + 1, p)
    p += 8 * (int(nrows) + 1)
    runs = np.frombuffer(raw, np.uint32, total, p)
    assert p + 4 * total == len(raw)
    return targets, off, runs


def _read_move_bucket(path):
    """The compact bucket layouts of csrc/cpd_io.cpp (MoveBucketFile): DOSCPD02
    (rows after the header) or DOSCPD03 (rows striped over part files
    {path}.{fingerprint:016x}.p{j}: unit u of stripe_rows rows is unit u // K of
    part u % K)."""
    raw = open(path, "rb").read()
    assert raw[:8] in (b"DOSCPD02", b"DOSCPD03")
    n, nrows, bid, method, key, maxworker, words, bits = (int(x) for x in np.frombuffer(raw, np.uint32, 8, 8))
    assert bits in (1, 2, 4) and words == (n * bits + 31) // 32
    total = int(np.frombuffer(raw, np.uint64, 1, 40)[0])
    if raw[:8] == b"DOSCPD02":
        p = 56
        targets = np.frombuffer(raw, np.uint32, nrows, p)
        counts = np.frombuffer(raw, np.uint32, nrows, p + 4 * nrows)
        rows_at = -(-(p + 8 * nrows) // 4096) * 4096
        assert len(raw) == rows_at + 4 * words * nrows
        moves = np.frombuffer(raw, np.uint32, nrows * words, rows_at).reshape(nrows, words)
    else:
        K, S = (int(x) for x in np.frombuffer(raw, np.uint32, 2, 56))
        p = 64
        targets = np.frombuffer(raw, np.uint32, nrows, p)
        counts = np.frombuffer(raw, np.uint32, nrows, p + 4 * nrows)
        assert len(raw) == p + 8 * nrows
        fp = int(np.frombuffer(raw, np.uint64, 1, 48)[0])
        parts = [np.fromfile(f"{path}.{fp:016x}.p{j}", np.uint32).reshape(-1, words)
                 for j in range(K)]
        moves = np.empty((nrows, words), np.uint32)
        for u in range(-(-nrows // S)):
            r0, r1 = u * S, min(nrows, u * S + S)
            q = (u // K) * S
            moves[r0:r1] = parts[u % K][q:q + (r1 - r0)]
        assert sum(len(x) for x in parts) == nrows
    assert int(counts.sum()) == total
    return targets, counts, moves, bits


@pytest.mark.parametrize("fmt", ["moves", "moves1", "rle"])
@pytest.mark.parametrize("method,key", [("mod", 5), ("div", 7)])
def test_make_cpd_auto_pipeline_matches_sequential(tmp_path, method, key, fmt):
    """The overlapped writer (build block k+1 while a pool copies block k out
    of HBM and writes it in place) gives byte-identical bucket files to the
    sequential path, in every layout (move tables striped over part files,
    DOSCPD03, the default; in one file, DOSCPD02, --stripes 1; DOSCPD01 run
    words); with --batch 1024 the blocks straddle bucket boundaries and
    --write-threads 3 interleaves pieces of several buckets."""
    prefix = str(tmp_path / "g")
    subprocess.run([os.path.join(BIN, "gen_synth"), "--width", "64", "--height", "48", "--seed",
                    "5", "--out", prefix, "--queries", "10"], check=True, capture_output=True)
    xy = prefix + ".xy"
    dirs = {}
    # "reserve": the auto batch above a 1-GiB HBM reserve (cpd_graph_set_hbm_reserve)
    for mode, extra in [("seq", ["--no-pipeline", "--batch", "1024"]),
                        ("pipe", ["--write-threads", "3", "--batch", "1024"]),
                        ("reserve", ["--hbm-reserve", "1"]), ("too_much", ["--hbm-reserve", "1e7"])]:
        out = str(tmp_path / mode)
        p = subprocess.run([os.path.join(BIN, "make_cpd_auto"), "--input", xy, "--partmethod",
                            method, "--partkey", str(key), "--workerid", "1", "--maxworker", "2",
                            "--outdir", out, "--device", "0",
                            "--format", "rle" if fmt == "rle" else "moves",
                            "--stripes", "1" if fmt == "moves1" else "16",
                            "--plan", str(tmp_path / "g.plan")] + extra,
                           capture_output=True, text=True, timeout=300)
        if mode == "too_much":  # a reserve past the free HBM: refused, nothing built
            assert p.returncode != 0 and "HBM reserve" in p.stderr, p.stderr
            continue
        assert p.returncode == 0, p.stderr
        dirs[mode] = out
    seq = sorted(f for f in os.listdir(dirs["seq"]) if f.endswith(".cpd"))
    pipe = sorted(f for f in os.listdir(dirs["pipe"]) if f.endswith(".cpd"))
    assert seq == pipe and len(seq) == key // 2
    assert not [f for f in os.listdir(dirs["pipe"]) if f.endswith(".tmp")]
    assert sorted(f for f in os.listdir(dirs["reserve"]) if f.endswith(".cpd")) == seq
    files = sorted(f for f in os.listdir(dirs["seq"]) if ".cpd" in f)  # with the parts
    assert files == sorted(f for f in os.listdir(dirs["pipe"]) if ".cpd" in f)
    assert (len(files) > len(seq)) == (fmt == "moves")
    for f in files:
        a = open(os.path.join(dirs["seq"], f), "rb").read()
        b = open(os.path.join(dirs["pipe"], f), "rb").read()
        assert a == b, f
        assert open(os.path.join(dirs["reserve"], f), "rb").read() == a, f
    # one bucket against the CPU oracle
    g = cpd.synth_road_graph(64, 48, seed=5)
    order = oracle.dfs_preorder(g.row_ptr, g.dst)
    if fmt == "rle":
        targets, off, runs = _read_bucket(os.path.join(dirs["pipe"], pipe[0]))
        o_off, o_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, np.array(targets))
        np.testing.assert_array_equal(off, o_off)
        np.testing.assert_array_equal(runs, o_runs)
    else:
        targets, counts, moves, bits = _read_move_bucket(os.path.join(dirs["pipe"], pipe[0]))
        assert bits == 2  # out-degrees <= 4
        o_off, o_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, np.array(targets))
        np.testing.assert_array_equal(counts, np.diff(o_off))
        np.testing.assert_array_equal(moves, oracle.moves_from_runs(o_off, o_runs, g.n, bits))
