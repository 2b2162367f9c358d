"""The hierarchy contracted on the GPU (ch_gpu.cpp / ch_kernels.hip) is the
host build's (ch.cpp), rank for rank and arc for arc: same priorities, same
independent sets, same witness-search cut-offs (the GPU heap replays
libstdc++'s push_heap / pop_heap), same shortcut merges.  Every array the
plan exports is compared; rows built from either plan are then the same by
construction (they are a function of exact distances in any case)."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import cpd
from graphs import GRAPHS

KEYS = ("rank", "up_off", "up_dst", "up_w", "dn_off", "dn_dst", "dn_w", "level_up", "level_dn")


def same_hierarchy(a, b):
    for k in KEYS:
        assert np.array_equal(a[k], b[k]), k


def test_ch_gpu_needs_a_gpu():
    """Without a visible GPU the GPU contraction fails loudly (no silent host
    build behind the flag)."""
    if cpd.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(cpd.CpdError):
        cpd.Plan(GRAPHS["synth"](), gpu=0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_ch_gpu_identical_small(name):
    g = GRAPHS[name]()
    same_hierarchy(cpd.Plan(g).export_ch(), cpd.Plan(g, gpu=0).export_ch())


@pytest.mark.gpu
@pytest.mark.parametrize("settle", [0, 20, 3])
def test_ch_gpu_identical_settle_limits(settle):
    """Small settle limits cut many witness searches short: the cut must fall
    at the same settled node on both sides."""
    g = cpd.synth_road_graph(120, 90, seed=3)
    same_hierarchy(cpd.Plan(g, settle=settle).export_ch(),
                   cpd.Plan(g, settle=settle, gpu=0).export_ch())


@pytest.mark.gpu
def test_ch_gpu_identical_spec_graph():
    g = cpd.synth_road_graph(160, 160, seed=4, style="spec")
    same_hierarchy(cpd.Plan(g).export_ch(), cpd.Plan(g, gpu=0).export_ch())


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"CPD_CH_WS": "16,8,2"},
                                 {"CPD_CH_WS": "16,8,2", "CPD_CH_NOWAVE": "1"},
                                 {"CPD_CH_WAVE": "0"}, {"CPD_CH_WAVE": "1000000000"},
                                 {"CPD_CH_WAVE": "1000000000", "CPD_CH_TINY": "0"}])
def test_ch_gpu_search_routes(env):
    """Every route a witness search can take — the lane workspace (here tiny,
    so most searches overflow it), the wave kernel's LDS, the large HBM
    workspace sized from the largest degree — gives the same hierarchy."""
    code = (
        "import sys; sys.path[:0] = %r\n"
        "import numpy as np, cpd\n"
        "g = cpd.synth_road_graph(80, 60, seed=9)\n"
        "a = cpd.Plan(g).export_ch(); b = cpd.Plan(g, gpu=0).export_ch()\n"
        "assert all(np.array_equal(a[k], b[k]) for k in a), 'differs'\n"
        "print('ok')\n" % (sys.path[:3],))
    env = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


@pytest.mark.gpu
def test_ch_gpu_identical_1m():
    """configs[3]'s graph (1000 x 1000, the bench workload): identical
    hierarchy, and the GPU build's time next to the host's."""
    g = cpd.synth_road_graph(1000, 1000, seed=1)
    t = time.time()
    b = cpd.Plan(g, gpu=0)
    t_gpu = time.time() - t
    t = time.time()
    a = cpd.Plan(g)
    t_host = time.time() - t
    print(f"\n1M CH: host {t_host:.2f} s ({a.info()['ch_seconds']:.2f} s CH), "
          f"GPU {t_gpu:.2f} s ({b.info()['ch_seconds']:.2f} s CH)")
    same_hierarchy(a.export_ch(), b.export_ch())


@pytest.mark.gpu
def test_make_cpd_auto_ch_gpu_and_host_same_files(tmp_path):
    """The drop-in executable: a worker whose plan is contracted on its GPU
    (the default) and one told --ch-host write byte-identical bucket files
    and column order, and save the same plan."""
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    binp = os.path.join(root, "bin")
    prefix = str(tmp_path / "g")
    subprocess.run([os.path.join(binp, "gen_synth"), "--width", "60", "--height", "50", "--seed",
                    "3", "--out", prefix], check=True, capture_output=True, timeout=120)
    digests = {}
    for mode in ("gpu", "host"):
        out = tmp_path / mode
        out.mkdir()
        cmd = [os.path.join(binp, "make_cpd_auto"), "--input", prefix + ".xy", "--partmethod",
               "div", "--partkey", "4", "--workerid", "1", "--maxworker", "4", "--outdir",
               str(out), "--device", "0", "--plan", str(out / "g.plan")]
        if mode == "host":
            cmd.append("--ch-host")
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        files = sorted(f for f in os.listdir(out) if ".cpd" in f or f.endswith(".order"))
        assert any(f.endswith(".cpd") for f in files)
        digests[mode] = {f: hashlib.sha256(open(out / f, "rb").read()).hexdigest() for f in files}
        a = cpd.Plan.load(str(out / "g.plan")).export_ch()
        digests[mode]["plan"] = hashlib.sha256(
            b"".join(np.ascontiguousarray(a[k]).tobytes() for k in KEYS)).hexdigest()
    assert digests["gpu"] == digests["host"]
