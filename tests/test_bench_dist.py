"""The N > 1 bench path on CPU: two gloo ranks run bench.py's sharding and
aggregation (Comm, shard_targets, batch_of, assemble) around a stand-in
compute step, and rank 0's line is checked."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import numpy as np
import torch.distributed as dist
import bench

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
args = bench.parse(["--steps", "3", "--warmup", "1", "--width", "40", "--partkey", "8",
                    "--batch", "1024"])
comm = bench.Comm(world, rank, rank, device=None)
n = 40 * 40
owned = bench.shard_targets(n, world, args.partmethod, args.partkey, rank)
seen = [bench.batch_of(owned, 1024, i) for i in range(args.warmup + args.steps)]
comm.barrier()
t0 = time.perf_counter()
time.sleep(0.05 * (rank + 1))            # uneven ranks: max must win
elapsed = time.perf_counter() - t0
(emax,) = comm.reduce([elapsed], "MAX")
ranks = bench.rank_table(1024, args.steps, [v[0] for v in comm.gather([elapsed])])
qt = comm.reduce([1000.0, 10.0 * (rank + 1), 5000.0], "SUM")
(qmax,) = comm.reduce([10.0 * (rank + 1)], "MAX")
allowned = [None] * world
dist.all_gather_object(allowned, owned.tolist())
if rank == 0:
    out = bench.assemble(args, world, (n, 4000), 1024, emax, qt, qmax, 1024, 2048, {}, None,
                         None, None)
    out["ranks"] = ranks
    out["_owned"] = allowned
    out["_elapsed_local"] = elapsed
    print("RESULT " + json.dumps(out), flush=True)
dist.destroy_process_group()
'''


def test_two_rank_gloo_aggregation(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port",
                        "29631", str(script)], capture_output=True, text=True, env=env,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][0]
    out = json.loads(line[len("RESULT "):])
    # the two shards are disjoint and cover every node (div 8 over 2 workers)
    owned = out.pop("_owned")
    assert sorted(owned[0] + owned[1]) == list(range(1600))
    assert not set(owned[0]) & set(owned[1])
    # value uses the MAX elapsed over ranks and counts both ranks' rows
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    emax = 3 * 1024 * 2 / out["value"]
    assert emax >= 0.099  # rank 1 slept 0.1 s
    assert out["queries_per_s"] == pytest.approx(2000.0 / 0.020, rel=1e-6)
    # the per-rank view: rank 1 slept twice as long and limits the line
    rk = out["ranks"]
    assert [r["rank"] for r in rk["per_rank"]] == [0, 1] and rk["slowest_rank"] == 1
    assert rk["per_rank"][1]["ms_per_step"] > rk["per_rank"][0]["ms_per_step"]
    assert rk["imbalance_max_over_min"] > 1.5
    assert rk["per_rank"][1]["ms_per_step"] == pytest.approx(emax / 3 * 1e3, rel=1e-3)
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "higher_is_better",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out


FB_WORKER = r'''
import json, os, sys, time, types
sys.path.insert(0, os.environ["ROOT"])
import bench

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
cache = os.environ["CACHE"]
args = bench.parse(["--width", "40", "--cache", cache])
filecomm = os.environ.get("FILECOMM") == "1"
if filecomm:  # what --full-build-only runs: no torch in the ranks
    comm = bench.FileComm(world, rank, rank, os.path.join(cache, "comm"))
else:
    import torch.distributed as dist
    dist.init_process_group("gloo")
    comm = bench.Comm(world, rank, rank, device=None)
if rank == 0:  # a stale directory from an earlier run, with a stale plan cache
    stale = bench.full_build_dir(args, world)
    os.makedirs(stale, exist_ok=True)
    open(os.path.join(stale, "stale.plan"), "w").write("old")
seen = {}

def fake_make_cpd_auto(cmd, **kw):
    """Stands in for bin/make_cpd_auto: records what it was asked to do."""
    a = dict(zip(cmd[1::2], cmd[2::2]))
    outdir = a["--outdir"]
    seen.update(cmd=cmd, dir_entries=sorted(os.listdir(outdir)), t=time.time())
    wid = int(a["--workerid"])
    if "--discard" not in cmd:
        open(os.path.join(outdir, f"g-div-8-{wid}.cpd"), "wb").write(b"x" * 1000)
    rec = {"worker": wid, "maxworker": int(a["--maxworker"]), "rows": 100 + wid, "runs": 1000,
           "export_bytes": 5000, "export_span_s": 0.5, "total_s": 1.0 + 0.25 * wid}
    return types.SimpleNamespace(returncode=0, stdout="make_cpd_auto-json: " + json.dumps(rec),
                                 stderr="")

fb, rec = bench.full_build_leg(args, "/nonexistent.xy", world, rank, 0, comm,
                               runner=fake_make_cpd_auto)
mine = {"cmd": seen["cmd"], "entries": seen["dir_entries"]}
if filecomm:
    allseen = comm._exchange(mine)
    assert "torch" not in sys.modules  # the ranks never load torch (nor HIP)
else:
    allseen = [None] * world
    dist.all_gather_object(allseen, mine)
if rank == 0:
    print("RESULT " + json.dumps({"fb": fb, "seen": allseen}), flush=True)
if not filecomm:
    dist.destroy_process_group()
'''


@pytest.mark.parametrize("filecomm", [False, True], ids=["gloo", "filecomm"])
def test_eight_rank_full_build_plumbing(tmp_path, filecomm):
    """The end-to-end worker leg at 8 ranks on gloo (the driver's N = 8
    scaling run, rehearsed on CPU): every rank runs worker r of the div-8
    partition only after rank 0 has replaced the stale output directory
    (no rank may see the old plan cache), rank 0 writes files
    and the others --discard, and the node's figures aggregate all ranks."""
    script = tmp_path / "fb.py"
    script.write_text(FB_WORKER)
    env = dict(os.environ, ROOT=ROOT, CACHE=str(tmp_path / "cache"), MASTER_ADDR="127.0.0.1",
               OMP_NUM_THREADS="1", FILECOMM="1" if filecomm else "0")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=8", "--master-addr", "127.0.0.1", "--master-port",
                        "29634" if filecomm else "29633", str(script)], capture_output=True,
                       text=True, env=env,
                       timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][0]
    out = json.loads(line[len("RESULT "):])
    fb, seen = out["fb"], out["seen"]
    for r, sv in enumerate(seen):
        cmd = sv["cmd"]
        a = dict(zip(cmd[1::2], cmd[2::2]))
        assert a["--workerid"] == str(r) and a["--maxworker"] == "8"
        assert a["--partmethod"] == "div" and a["--partkey"] == "8" and a["--format"] == "moves"
        assert ("--discard" in cmd) == (r != 0)
        assert "stale.plan" not in sv["entries"]  # the cold directory, never the stale one
    assert fb["total_s"] == 1.0 + 0.25 * 7           # the slowest worker
    assert fb["rows"] == sum(100 + r for r in range(8))
    assert fb["export_GB"] == round(8 * 5000 / 1e9, 2)
    assert fb["files_GB"] == round(1000 / 1e9, 2)    # rank 0's files
    # each worker's own line; the slowest one named
    assert [p["worker"] for p in fb["per_rank"]] == list(range(8))
    assert [p["total_s"] for p in fb["per_rank"]] == [1.0 + 0.25 * r for r in range(8)]
    assert fb["per_rank"][3]["rows_per_s"] == round(103 / 1.75, 1)
    assert fb["slowest_rank"] == 7 and fb["imbalance_max_over_min"] == round(2.75 / 1.0, 4)
