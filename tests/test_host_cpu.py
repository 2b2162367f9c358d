"""Host-side logic of libcpd on CPU: partitioner, column order, contraction
hierarchy (checked by a numpy PHAST against the oracle's Dijkstra), plan
persistence, synthetic generators, the C ABI's exported symbols, and that GPU
entry points fail loudly without a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components

import cpd
import oracle
from graphs import GRAPHS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_abi_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "cpd_api.h")).read()
    declared = set(re.findall(r"\b(cpd_[a-z_]+)\s*\(", hdr))
    assert len(declared) > 30
    missing = [s for s in sorted(declared) if not hasattr(cpd.lib, s)]
    assert not missing, missing
    assert set(cpd.EXPORTED) == declared
    assert "gfx950" in cpd.version()


def test_library_built_from_this_tree():
    """Build provenance: the hash libcpd.so embeds (Makefile SRC_SHA) equals the
    hash of the sources shipped beside it."""
    assert cpd.lib_src_sha() == cpd.src_sha()


@pytest.mark.parametrize("method", ["mod", "div"])
def test_partition_matches_oracle(method):
    rng = np.random.default_rng(1)
    for _ in range(200):
        n = int(rng.integers(1, 5000))
        W = int(rng.integers(1, 12))
        key = int(rng.integers(1, 300))
        node = int(rng.integers(0, n))
        assert cpd.partition(n, W, method, key, node) == oracle.partition(n, W, method, key, node)
    # owned_nodes (vectorised) agrees with the per-node function
    n, W, key = 1000, 3, 7
    for w in range(W):
        own = cpd.owned_nodes(n, W, method, key, w)
        ref = [v for v in range(n) if oracle.partition(n, W, method, key, v)[0] == w]
        assert own.tolist() == ref


def test_partition_errors():
    with pytest.raises(cpd.CpdError):
        cpd.partition(10, 2, "mod", 0, 1)
    with pytest.raises(cpd.CpdError):
        cpd.partition(10, 2, "mod", 3, 10)
    with pytest.raises(cpd.CpdError):
        cpd.partition(10, 2, "range", 3, 1)


def test_dfs_order_matches_oracle():
    for name, f in GRAPHS.items():
        g = f()
        a = cpd.dfs_preorder(g.row_ptr, g.dst)
        b = oracle.dfs_preorder(g.row_ptr, g.dst)
        assert np.array_equal(a, b), name
        assert np.array_equal(np.sort(a), np.arange(g.n))


def _phast(ch, n, t):
    INF = np.uint64(1) << np.uint64(62)
    d = np.full(n, INF, np.uint64)
    lu, ld = ch["level_up"], ch["level_dn"]
    dn_off, dn_dst, dn_w = ch["dn_off"].astype(np.int64), ch["dn_dst"], ch["dn_w"].astype(np.uint64)
    up_off, up_dst, up_w = ch["up_off"].astype(np.int64), ch["up_dst"], ch["up_w"].astype(np.uint64)
    for lvl in range(int(lu.max()) + 1):
        for v in np.nonzero(lu == lvl)[0]:
            best = np.uint64(0) if v == t else INF
            a, b = dn_off[v], dn_off[v + 1]
            if b > a:
                best = min(best, (d[dn_dst[a:b]] + dn_w[a:b]).min())
            d[v] = best
    for lvl in range(int(ld.max()) + 1):
        for v in np.nonzero(ld == lvl)[0]:
            a, b = up_off[v], up_off[v + 1]
            if b > a:
                d[v] = min(d[v], (d[up_dst[a:b]] + up_w[a:b]).min())
    d[d >= INF] = oracle.INF
    return d.astype(np.uint32)


@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_hierarchy_sweeps_give_exact_distances(name):
    g = GRAPHS[name]()
    plan = cpd.Plan(g, threads=2)
    ch = plan.export_ch()
    rank = ch["rank"]
    assert np.array_equal(np.sort(rank), np.arange(g.n))
    # up arcs climb, down arcs descend, levels respect the sweep order
    tails_up = np.repeat(np.arange(g.n), np.diff(ch["up_off"].astype(np.int64)))
    tails_dn = np.repeat(np.arange(g.n), np.diff(ch["dn_off"].astype(np.int64)))
    assert np.all(rank[ch["up_dst"]] > rank[tails_up])
    assert np.all(rank[ch["dn_dst"]] < rank[tails_dn])
    assert np.all(ch["level_up"][ch["dn_dst"]] < ch["level_up"][tails_dn])
    assert np.all(ch["level_dn"][ch["up_dst"]] < ch["level_dn"][tails_up])
    rng = np.random.default_rng(2)
    for t in rng.choice(g.n, size=min(g.n, 6), replace=False):
        ref = oracle.reverse_dijkstra(g.row_ptr, g.dst, g.w, t)
        np.testing.assert_array_equal(_phast(ch, g.n, t), ref, err_msg=f"{name} t={t}")


def test_hierarchy_is_deterministic_across_threads():
    g = cpd.synth_road_graph(30, 30, seed=4)
    a = cpd.Plan(g, threads=1).export_ch()
    b = cpd.Plan(g, threads=4).export_ch()
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_plan_save_load_roundtrip(tmp_path):
    g = cpd.synth_road_graph(20, 15, seed=2)
    p = cpd.Plan(g)
    path = str(tmp_path / "g.plan")
    p.save(path)
    q = cpd.Plan.load(path)
    assert p.info() == q.info()
    assert np.array_equal(p.order(), q.order())
    a, b = p.export_ch(), q.export_ch()
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    with open(path, "r+b") as f:
        f.write(b"garbage!")
    with pytest.raises(cpd.CpdError):
        cpd.Plan.load(path)


def test_plan_rejects_bad_graphs():
    # out-degree 16 exceeds the 4-bit move field
    rp = np.array([0, 16] + [16] * 16, np.uint32)
    dst = np.arange(1, 17, dtype=np.uint32)
    g = cpd.RoadGraph(rp, dst, np.ones(16, np.uint32))
    with pytest.raises(cpd.CpdError) as e:
        cpd.Plan(g)
    assert e.value.code == cpd.CPD_E_RANGE
    # distances that could reach 2^32-1
    rp = np.array([0, 1, 2, 2], np.uint32)
    g = cpd.RoadGraph(rp, np.array([1, 2], np.uint32), np.array([0xF0000000, 0x20000000], np.uint32))
    with pytest.raises(cpd.CpdError) as e:
        cpd.Plan(g)
    assert e.value.code == cpd.CPD_E_RANGE
    # malformed CSR
    with pytest.raises(cpd.CpdError):
        cpd.Plan(cpd.RoadGraph(np.array([0, 2], np.uint32), np.array([5], np.uint32),
                               np.array([1], np.uint32)))


def test_synthetic_graph_properties():
    g = cpd.synth_road_graph(60, 50, seed=1)
    h = cpd.synth_road_graph(60, 50, seed=1)
    assert np.array_equal(g.dst, h.dst) and np.array_equal(g.w, h.w)
    assert g.n == 3000 and abs(g.m / g.n - 2.5) < 0.01
    deg = np.diff(g.row_ptr.astype(np.int64))
    assert deg.max() <= 4 and g.w.min() >= 1 and g.w.max() <= 65535
    rows = np.repeat(np.arange(g.n), deg)
    A = csr_matrix((np.ones(g.m), (rows, g.dst)), shape=(g.n, g.n))
    ncomp, _ = connected_components(A, directed=True, connection="strong")
    assert ncomp == 1
    wc = cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3)
    changed = wc != g.w
    assert 0.05 < changed.mean() < 0.15 and np.all(wc >= g.w) and np.all(wc <= 3 * g.w + 1)


def test_gpu_entry_points_fail_loudly_without_gpu():
    if cpd.device_count() > 0:
        pytest.skip("a GPU is present")
    g = cpd.synth_road_graph(5, 5, seed=1)
    with pytest.raises(cpd.CpdError) as e:
        cpd.Graph(cpd.Plan(g))
    assert e.value.code == cpd.CPD_E_HIP and "no CPU fallback" in str(e.value)
    with pytest.raises(cpd.CpdError) as e:
        cpd.device_mem_info(0)
    assert e.value.code == cpd.CPD_E_HIP


def test_tools_roundtrip_and_fail_loudly(tmp_path):
    prefix = str(tmp_path / "s")
    subprocess.run([os.path.join(ROOT, "bin", "gen_synth"), "--width", "8", "--height", "6",
                    "--seed", "3", "--out", prefix, "--queries", "20"], check=True,
                   capture_output=True)
    g = cpd.synth_road_graph(8, 6, seed=3)
    lines = open(prefix + ".xy").read().splitlines()
    assert lines[3] == f"nodes {g.n} edges {g.m}"
    e = [tuple(map(int, ln.split()[1:])) for ln in lines if ln.startswith("e ")]
    tails = np.repeat(np.arange(g.n), np.diff(g.row_ptr.astype(np.int64)))
    assert e == list(zip(tails.tolist(), g.dst.tolist(), g.w.tolist()))
    if cpd.device_count() == 0:
        p = subprocess.run([os.path.join(ROOT, "bin", "make_cpd_auto"), "--input", prefix + ".xy",
                            "--partmethod", "mod", "--partkey", "2", "--workerid", "0",
                            "--maxworker", "2", "--outdir", str(tmp_path / "idx")],
                           capture_output=True, text=True)
        assert p.returncode != 0 and "no GPU" in p.stderr


def test_space_preflight_library():
    """cpd_bucket_bytes / cpd_space_check (make_cpd_auto's disk preflight):
    the row bytes of a worker's compact buckets, and CPD_E_IO with the numbers
    when a tmpfs cannot hold them."""
    # 1M nodes at 2 bits: 62500 words per row; + target and count per row
    b = cpd.bucket_bytes(1_000_000, 2, 125_000, nbuckets=1, stripes=16)
    assert b == 125_000 * (4 * 62_500 + 8) + 17 * 4096
    assert cpd.bucket_bytes(10, 1, 0, nbuckets=2, stripes=1) == 2 * 2 * 4096
    free = cpd.space_check("/dev/shm", 1)
    assert free > 0
    with pytest.raises(cpd.CpdError) as e:
        cpd.space_check("/dev/shm", free + (1 << 40))
    assert "error -6" in str(e.value) and "MiB free" in str(e.value)
    with pytest.raises(cpd.CpdError):
        cpd.space_check("/no/such/dir/for/cpd", 1)


def test_make_cpd_auto_refuses_a_disk_too_small(tmp_path):
    """A worker whose bucket files outgrow --outdir (a tmpfs here) exits with
    status 3 and a one-line message before any plan or GPU work — not with a
    write error minutes in."""
    shm = "/dev/shm"
    free = os.statvfs(shm).f_bavail * os.statvfs(shm).f_frsize
    # one worker owning every row: n^2 / 4 bytes at 2 bits per column
    width = int(np.ceil(np.sqrt(np.sqrt(6.0 * free))))
    if width > 1400:
        pytest.skip(f"{shm} has {free >> 30} GiB free: the graph would be too large")
    prefix = str(tmp_path / "big")
    subprocess.run([os.path.join(ROOT, "bin", "gen_synth"), "--width", str(width), "--height",
                    str(width), "--seed", "4", "--out", prefix], check=True,
                   capture_output=True, timeout=300)
    out = os.path.join(shm, f"cpd_preflight_{os.getpid()}")
    try:
        p = subprocess.run([os.path.join(ROOT, "bin", "make_cpd_auto"), "--input", prefix + ".xy",
                            "--partmethod", "div", "--partkey", "1", "--workerid", "0",
                            "--maxworker", "1", "--outdir", out],
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
        msg = p.stderr.strip().splitlines()
        assert len(msg) == 1 and "MiB free" in msg[0] and "need" in msg[0], p.stderr
        assert not [f for f in os.listdir(out) if f.endswith(".plan") or ".cpd" in f]
    finally:
        subprocess.run(["rm", "-rf", out])
