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
qt = comm.reduce([1000.0, 10.0 * (rank + 1), 5000.0], "SUM")
(qmax,) = comm.reduce([10.0 * (rank + 1)], "MAX")
allowned = [None] * world
dist.all_gather_object(allowned, owned.tolist())
if rank == 0:
    out = bench.assemble(args, world, (n, 4000), 1024, emax, qt, qmax, 1024, 2048, {}, None,
                         None, None)
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
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "higher_is_better",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out
