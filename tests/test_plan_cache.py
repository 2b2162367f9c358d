"""Plan cache under concurrent workers (host only, no GPU).

make_cpds.py:58-60 starts every worker's make_cpd_auto at once (tmux -d) on
one --outdir.  With a cold cache each would build the same hierarchy and save
it; cpd_plan_cache serialises that with an flock so one builds, the others
wait and load its file, and no save can truncate another's temporary."""
import glob
import os
import subprocess

import numpy as np
import pytest

import cpd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def _gen(tmp_path, w=160, seed=4):
    prefix = str(tmp_path / "g")
    subprocess.run([os.path.join(BIN, "gen_synth"), "--width", str(w), "--seed", str(seed),
                    "--out", prefix, "--queries", "10"], check=True, capture_output=True)
    return prefix + ".xy"


def test_concurrent_cold_cache_one_builder(tmp_path):
    xy = _gen(tmp_path)
    outdir = str(tmp_path / "index")
    W = 3
    procs = [subprocess.Popen([os.path.join(BIN, "make_cpd_auto"), "--input", xy, "--partmethod",
                               "mod", "--partkey", "3", "--workerid", str(wid), "--maxworker",
                               str(W), "--outdir", outdir, "--plan-only", "--threads", "2"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for wid in range(W)]
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
    built = sum("built and cached" in o for o, _ in outs)
    loaded = sum("loaded plan" in o for o, _ in outs)
    assert built == 1 and loaded == W - 1, outs
    plans = glob.glob(os.path.join(outdir, "*.plan"))
    assert len(plans) == 1
    assert not glob.glob(os.path.join(outdir, "*.tmp*"))
    p = cpd.Plan.load(plans[0])
    assert p.info()["levels_up"] > 0


def test_cache_rebuilds_for_another_graph(tmp_path):
    g1 = cpd.synth_road_graph(30, 30, seed=1)
    g2 = cpd.synth_road_graph(30, 30, seed=2)
    path = str(tmp_path / "x.plan")
    p1, st1 = cpd.Plan.cache(path, g1)
    assert st1 == 1
    p1b, st1b = cpd.Plan.cache(path, g1)
    assert st1b == 0 and np.array_equal(p1.order(), p1b.order())
    p2, st2 = cpd.Plan.cache(path, g2)  # same path, other graph: rebuilt over it
    assert st2 == 1 and np.array_equal(p2.order(), cpd.Plan(g2).order())
    # a plan that cannot be saved is still returned (status 2)
    p3, st3 = cpd.Plan.cache(str(tmp_path / "no" / "such" / "dir" / "x.plan"), g1)
    assert st3 == 2 and p3.info()["n"] == g1.n


def _raw_plan(tmp_path):
    g = cpd.synth_road_graph(12, 10, seed=3)
    path = str(tmp_path / "p.plan")
    cpd.Plan(g).save(path)
    return g, path, bytearray(open(path, "rb").read())


def test_load_rejects_non_permutation_order(tmp_path):
    g, path, raw = _raw_plan(tmp_path)
    # layout: magic 8 | n m nlev_up nlev_dn (4 x u32) | bound u64 | seconds f64 |
    # vectors (u64 length + data): row_ptr, dst, w, order, ...
    pos = 8 + 16 + 16
    for _ in range(3):  # skip row_ptr, dst, w
        k = int(np.frombuffer(raw, np.uint64, 1, pos)[0])
        pos += 8 + 4 * k
    k = int(np.frombuffer(raw, np.uint64, 1, pos)[0])
    assert k == g.n
    order = np.frombuffer(raw, np.uint32, k, pos + 8).copy()
    order[1] = order[0]  # a duplicate column
    raw[pos + 8: pos + 8 + 4 * k] = order.tobytes()
    bad = str(tmp_path / "bad.plan")
    open(bad, "wb").write(bytes(raw))
    with pytest.raises(cpd.CpdError) as ei:
        cpd.Plan.load(bad)
    assert ei.value.code == cpd.CPD_E_IO and "permutation" in str(ei.value)


def test_load_rejects_truncated_hierarchy(tmp_path):
    g, path, raw = _raw_plan(tmp_path)
    bad = str(tmp_path / "trunc.plan")
    open(bad, "wb").write(bytes(raw[: len(raw) - 40]))
    with pytest.raises(cpd.CpdError) as ei:
        cpd.Plan.load(bad)
    assert ei.value.code == cpd.CPD_E_IO
