#!/usr/bin/env python3
"""bench.py — MI355X CPD build (sources/s, GTEPS) and table-search (queries/s).

Workloads (--workload; melb-both.xy is a missing blob, so every graph is the
seeded synthetic road graph of SURVEY.md §8d):
  synth1m (default, BASELINE.json configs[3]): 1000 x 1000 lattice (1M nodes,
    2.5M edges), seed 1, partition `div 8` over the ranks.  A step = one batch
    of --batch CPD rows built from the rank's own targets: two CH sweeps,
    first-move sets and the RLE rows, all resident in HBM (weak scaling: every
    rank builds the same number of rows per step; no collective on the data
    path).  Then 1M table-search queries against the rank's last batch.
  synth1m-spec: the same lattice with SURVEY.md §8d's recipe as written (node
    id = lattice cell, every edge bidirectional, out-edges E/N/W/S) instead
    of the shuffled ids / one-way streets / shuffled out-edge order.
  synth4m (configs[4]): 2000 x 2000, seed 4; 256k targets sampled (seed 5),
    `div 8`: rank r is worker r of 8 (one worker's ~32k rows per GPU, weak
    scaling).  Steps build batches of the worker's rows; then ALL its rows are
    streamed into a dense index and it serves its share of the 10M-query
    batch (t uniform over the sample, seed 6: ~1.25M routed to each worker).
  melb300k (configs[0]-[2] stand-in): 548 x 548 spec-style graph, seed 1,
    `mod 3`; query leg with the .diff stand-in as for synth1m.

One JSON line on rank 0: value = rows/s over all ranks; roofline for the
dominant build kernel from HIP events, query_roofline for the walk kernel;
cpu_baseline = the C oracle (OpenMP, all host threads of this job) on a
bounded sample of the same workload, plus the configs[0] partitioned run
(300k stand-in, mod 3: three workers one after another with every thread,
then at once with a third each), rank 0 at N = 1 only.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
  (N > 1 is launched by torch.distributed.run; RANK/LOCAL_RANK/WORLD_SIZE)
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "distributed-oracle-search_amd")
METRIC = "CPD build sources/sec + GTEPS; table-search queries/sec; % HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PLAN_TAG = "ch8212g"    # bump when the hierarchy builder changes (cache key)

WORKLOADS = {
    "synth1m": dict(width=1000, seed=1, style="shuffled", method="div", key=8, sample=None,
                    queries=1_000_000, config="configs[3]"),
    "synth1m-spec": dict(width=1000, seed=1, style="spec", method="div", key=8, sample=None,
                         queries=1_000_000, config="configs[3], SURVEY 8d recipe as written"),
    "synth4m": dict(width=2000, seed=4, style="shuffled", method="div", key=8,
                    sample=(262144, 5), queries=10_000_000, config="configs[4]"),
    "melb300k": dict(width=548, seed=1, style="spec", method="mod", key=3, sample=None,
                     queries=1_000_000, config="configs[0]-[2] stand-in"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="synth1m", choices=sorted(WORKLOADS))
    ap.add_argument("--width", type=int, default=0, help="override the lattice side")
    ap.add_argument("--seed", type=int, default=0, help="override the graph seed")
    ap.add_argument("--partmethod", default="")
    ap.add_argument("--partkey", type=int, default=0)
    ap.add_argument("--batch", type=int, default=0,
                    help="rows per step (multiple of 1024); 0 = what fits in HBM, <= 28672")
    ap.add_argument("--queries", type=int, default=0, help="0 = the workload's")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every host thread this job may use (OMP_NUM_THREADS or affinity)")
    ap.add_argument("--cpu-rows-per-thread", type=int, default=64,
                    help="CPU baseline sample: rows per host thread (~10 s of CPU work)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-cpu-partitioned", action="store_true",
                    help="skip the configs[0] mod-3 partitioned CPU run")
    ap.add_argument("--no-search", action="store_true", help="skip the cpd-search leg")
    ap.add_argument("--no-full-build", action="store_true",
                    help="skip the end-to-end worker build (make_cpd_auto, cold plan)")
    ap.add_argument("--full-build-discard", action="store_true",
                    help="full-build leg without file writes (make_cpd_auto --discard)")
    ap.add_argument("--full-build-only", action="store_true",
                    help="run only the end-to-end worker leg (no GPU context in the ranks)")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 --pmc passes that fill roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-worker", default="", help=argparse.SUPPRESS)
    ap.add_argument("--cache", default=os.environ.get("CPD_BENCH_CACHE", "/tmp/cpd-bench-cache"))
    a = ap.parse_args(argv)
    wl = WORKLOADS[a.workload]
    a.width = a.width or wl["width"]
    a.seed = a.seed or wl["seed"]
    a.style = wl["style"]
    a.partmethod = a.partmethod or wl["method"]
    a.partkey = a.partkey or wl["key"]
    a.sample = wl["sample"]
    a.queries = a.queries or wl["queries"]
    return a


def plan_path(args):
    style = "" if args.style == "shuffled" else f"-{args.style}"
    return os.path.join(args.cache, f"synth{args.width}-s{args.seed}{style}-{PLAN_TAG}.plan")


# rocprofv3 kernel names -> the library's timing names
KERNEL_NAMES = {"sweep_level<true": "sweep_up", "sweep_up_": "sweep_up",
                "sweep_level<false": "sweep_down", "sweep_down8": "sweep_down",
                "first_moves": "first_moves", "rle_scan<": "rle_count", "rle_emit": "rle_emit",
                "rle_moves": "rle_moves", "rle_count_ch": "rle_count", "rle_fix": "rle_fix",
                "moves_runs": "moves_runs", "DenseRows": "table_search_dense",
                "RleRows": "table_search", "table_search_dense": "table_search_dense",
                "table_search(": "table_search", "expand_rows": "expand_rows"}


def kernel_key(name):
    return next((v for k, v in KERNEL_NAMES.items() if k in name), None)


def pmc_traffic(args):
    """HBM traffic per launch from rocprofv3 PMC counters.

    One child run per counter (MI355X_MICROARCH.md: FETCH_SIZE costs 3 and
    WRITE_SIZE 2 of the 4 TCC slots, so they cannot share a pass), each a
    one-step build plus one dense query launch of the same workload.  Both
    counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
    16-B/lane streaming read, so it is doubled (the build kernels' loads are 16
    B per lane; the walk's 4-B and 16-B gathers are uncalibrated — the walk's
    read figure is reported raw x 2 as well, as an upper estimate); WRITE_SIZE
    is exact for 16-B stores.  Started before this process touches the GPU.
    Returns {name: {"launches", "read/write/bytes_per_launch"}} or None.
    """
    import csv
    import glob
    import shutil
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    out = {}
    base = tempfile.mkdtemp(prefix="pmc-", dir=args.cache)
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(base, counter)
        cmd = ["rocprofv3", "--pmc", counter, "-d", d, "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "1",
               "--warmup", "0", "--workload", args.workload, "--width", str(args.width),
               "--seed", str(args.seed), "--partmethod", args.partmethod, "--partkey",
               str(args.partkey), "--batch", str(args.batch), "--cache", args.cache]
        try:
            p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                               timeout=240, cwd=base)
        except subprocess.TimeoutExpired:
            log(f"pmc pass {counter} timed out")
            return None
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if p.returncode != 0 or not files:
            log(f"pmc pass {counter} failed: {p.stderr[-400:]}")
            return None
        for row in csv.DictReader(open(files[0])):
            name = kernel_key(row["Kernel_Name"])
            if name is None:
                continue
            e = out.setdefault(name, {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "n_FETCH_SIZE": 0,
                                      "n_WRITE_SIZE": 0})
            e[counter] += float(row["Counter_Value"])
            e["n_" + counter] += 1
    for e in out.values():
        nf, nw = max(1, e.pop("n_FETCH_SIZE")), max(1, e.pop("n_WRITE_SIZE"))
        e["launches"] = nf
        e["read_bytes_per_launch"] = 2.0 * e["FETCH_SIZE"] * 1024.0 / nf
        e["write_bytes_per_launch"] = e["WRITE_SIZE"] * 1024.0 / nw
        e["bytes_per_launch"] = e["read_bytes_per_launch"] + e["write_bytes_per_launch"]
    shutil.rmtree(base, ignore_errors=True)
    return out


def pmc_child(args):
    """One build step and one dense query launch under the profiler (no torch:
    nothing else on the GPU)."""
    sys.path.insert(0, PKG)
    import numpy as np
    import cpd
    plan = cpd.Plan.load(plan_path(args))
    n = plan.info()["n"]
    dev = cpd.Graph(plan, device=0, batch=args.batch)
    g = cpd.synth_road_graph(args.width, args.width, seed=args.seed, style=args.style)
    dev.set_coords(g.x, g.y)  # lane order as in the timed run
    owned = rank_targets(args, n, 1, 0)
    targets = batch_of(owned, dev.batch, 0)
    rows = dev.build_rows(targets)
    ix = cpd.Index.streamed(dev, targets, rows.count()[1], mode="dense")
    ix.append_rows(rows)
    del rows
    rng = np.random.default_rng(100)
    nq = min(args.queries, 1_000_000)
    ix.prepare(rng.integers(0, n, nq).astype(np.uint32), targets[rng.integers(0, len(targets), nq)])
    ix.run()


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# --------------------------------------------------------------------------
# distributed plumbing (importable; tests/test_bench_dist.py runs it on gloo)

class Comm:
    """Barrier / reductions over torch.distributed.  Only the bench harness
    uses them (timing and a handful of counters); nothing on the data path."""

    def __init__(self, world, rank, local, device=None, pg=None):
        self.world, self.rank, self.local, self.device = world, rank, local, device
        self.pg = world > 1 if pg is None else pg  # collectives through the process group

    def barrier(self):
        import torch
        if self.device is not None:
            torch.cuda.synchronize()
        if self.pg:
            import torch.distributed as dist
            dist.barrier()

    def reduce(self, vals, op):
        if not self.pg:
            return list(vals)
        import torch
        import torch.distributed as dist
        t = torch.tensor(vals, dtype=torch.float64, device=self.device or "cpu")
        dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
        return t.tolist()

    def gather(self, vals):
        """Every rank's `vals` (floats), in rank order."""
        if not self.pg:
            return [list(vals)]
        import torch
        import torch.distributed as dist
        t = torch.tensor(vals, dtype=torch.float64, device=self.device or "cpu")
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t)
        return [x.tolist() for x in out]


# The result line's file descriptor: stdout, or (with RCCL) a copy of it —
# RCCL prints its version banner on fd 1 when a communicator starts, so fd 1
# is pointed at stderr first and the one JSON line goes to the real stdout.
_RESULT_FD = None


def emit_line(line):
    sys.stdout.flush()
    os.write(_RESULT_FD if _RESULT_FD is not None else 1, (line + "\n").encode())


class FileComm:
    """Barrier / reductions through small files in a directory the node's
    ranks share — for --full-build-only, whose ranks then load neither torch
    nor HIP: on one shared GPU the workers' make_cpd_auto processes (and the
    launcher) are then the only processes holding the card."""

    def __init__(self, world, rank, local, path, timeout=1800.0):
        self.world, self.rank, self.local, self.device = world, rank, local, None
        self.path, self.timeout, self.gen = path, timeout, 0
        os.makedirs(path, exist_ok=True)

    def _exchange(self, vals):
        self.gen += 1
        mine = os.path.join(self.path, f"g{self.gen}.r{self.rank}")
        with open(mine + ".tmp", "w") as f:
            json.dump(vals, f)
        os.rename(mine + ".tmp", mine + ".json")
        names = [os.path.join(self.path, f"g{self.gen}.r{r}.json") for r in range(self.world)]
        deadline = time.time() + self.timeout
        while not all(os.path.exists(n) for n in names):
            if time.time() > deadline:
                raise RuntimeError(f"FileComm: ranks missing at step {self.gen} in {self.path}")
            time.sleep(0.05)
        out = []
        for n in names:
            with open(n) as f:
                out.append(json.load(f))
        return out

    def barrier(self):
        self._exchange(None)

    def reduce(self, vals, op):
        allv = self._exchange(list(vals))
        fn = {"SUM": sum, "MAX": max, "MIN": min}[op]
        return [fn(v[i] for v in allv) for i in range(len(vals))]

    def gather(self, vals):
        return [list(v) for v in self._exchange(list(vals))]


def rank_table(B, steps, elapsed):
    """The N > 1 line's per-rank view: each rank's step
    time and rows/s, and the spread — which rank limits the curve."""
    per = [{"rank": r, "ms_per_step": round(e / steps * 1e3, 3),
            "rows_per_s": round(B * steps / e, 1) if e else 0.0} for r, e in enumerate(elapsed)]
    lo, hi = min(elapsed), max(elapsed)
    return {"per_rank": per, "slowest_rank": max(range(len(elapsed)), key=lambda r: elapsed[r]),
            "imbalance_max_over_min": round(hi / lo, 4) if lo else None}


def shard_targets(nodenum, world, method, key, rank):
    """The rank's targets: distribution_controller partition, worker = rank."""
    sys.path.insert(0, PKG)
    import cpd
    return cpd.owned_nodes(nodenum, world, method, key, rank)


def sample_nodes(n, k, seed):
    """configs[4]'s sampled targets (without replacement), sorted."""
    import numpy as np
    return np.sort(np.random.default_rng(seed).choice(n, size=k, replace=False)).astype(np.uint32)


def rank_targets(args, n, world, rank):
    """synth1m / melb300k: the partition over `world` workers (rank = worker).
    synth4m: worker `rank` of the configuration's 8 over the sampled targets
    (one worker per GPU at any N: weak scaling)."""
    import numpy as np
    if args.sample is None:
        return shard_targets(n, world, args.partmethod, args.partkey, rank)
    s = sample_nodes(n, *args.sample).astype(np.int64)
    bid = s % args.partkey if args.partmethod == "mod" else s // (-(-n // args.partkey))
    return s[(bid % 8) == rank].astype(np.uint32)


def batch_of(owned, B, i):
    """Step i's targets: the next B of the rank's own, wrapping around."""
    import numpy as np
    idx = (np.arange(B, dtype=np.int64) + i * B) % len(owned)
    return owned[idx]


def assemble(args, world, graph_info, B, elapsed_max, q_totals, q_ms_max, nrows, nruns,
             kt, cpu, parity, pinfo, traffic=None):
    """Rank 0's JSON line.  value = rows built by ALL ranks / max rank time.
    roofline: the dominant kernel = the one moving the most algorithmic bytes
    (SURVEY.md §8d model, counted per launch by libcpd); achieved = those
    bytes / its summed event time; traffic = PMC bytes per launch of the same
    kernel (or None).  Not the kernel with the most device time: the next
    batch's up-sweep runs on its own stream beside this batch's first moves,
    and its ~190 small latency-bound launches wait there behind the first
    moves' workgroups (summed, ~31 ms of events per step for ~10 GB), so
    event time would name a kernel that is stretched, not heavy."""
    n, m = graph_info
    total_rows = world * args.steps * B
    value = total_rows / elapsed_max
    roof = None
    if kt:
        name, k = max(((a, b) for a, b in kt.items() if a not in _COUNTERS),
                      key=lambda kv: kv[1]["bytes"])
        achieved = k["bytes"] / (k["ms"] / 1e3) / 1e9 if k["ms"] > 0 else 0.0
        t = (traffic or {}).get(name)
        roof = {"bound": "hbm", "kernel": name, "chosen_by": "most algorithmic bytes",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": round(t["bytes_per_launch"], 1) if t else None,
                "traffic_unit": "bytes/launch (PMC: 2*FETCH_SIZE + WRITE_SIZE, KiB->B)",
                "traffic_scope": ("rank 0's GPU, one step of its own targets (every rank "
                                  "builds the same batch shape)" if world > 1 else "this GPU")
                if t else "not collected (--no-pmc, no rocprofv3, or a shared-GPU rehearsal)",
                "launches": k["launches"],
                "avg_launch_us": round(k["ms"] * 1e3 / max(1, k["launches"]), 3),
                "bytes_per_launch": round(k["bytes"] / max(1, k["launches"]), 1)}
    qps = q_totals[0] / (q_ms_max / 1e3) if q_ms_max > 0 else 0.0
    wl = WORKLOADS[getattr(args, "workload", "synth1m")]
    return {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "sources/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded grid-perturbed road graph; melb-both.xy blob is missing)",
        "config": {"workload": f"synthetic-{n // 1000}k-road cpd-build {args.partmethod} "
                               f"{args.partkey} + table-search",
                   "baseline_config": wl["config"],
                   "graph": f"grid-perturbed {args.width}x{args.width} seed {args.seed} "
                            f"({getattr(args, 'style', 'shuffled')})",
                   "nodes": n, "edges": m, "rows_per_step_per_gpu": B,
                   "partition": f"{args.partmethod} {args.partkey}",
                   "parallelism": f"target-partition x{world} (no collective)"},
        "gteps": round(value * m / 1e9, 3),
        "queries_per_s": round(qps, 1),
        "query_mean_moves": round(q_totals[2] / max(1.0, q_totals[0]), 1),
        "mean_runs_per_row": round(nruns / max(1, nrows), 1),
        "roofline": roof,
        "cpu_baseline": cpu,
        "parity_sample_bit_exact": parity,
        "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                        "GBps": round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1) if v["ms"] else 0}
                    for k, v in (kt or {}).items() if k not in _COUNTERS},
        # narrow distance rows: 256-target groups kept wide (u32) / all groups
        "narrow_rows": {"wide_groups": (kt or {}).get("wide_rows", {}).get("launches"),
                        "groups": (kt or {}).get("group_rows", {}).get("launches")},
        # first-move buffer sets the emit overlap rotates through (libcpd kSets)
        "emit_sets": (kt or {}).get("emit_sets", {}).get("launches"),
        "hierarchy": {"arcs": pinfo["ch_up_arcs"] + pinfo["ch_dn_arcs"],
                      "levels": [pinfo["levels_up"], pinfo["levels_dn"]],
                      "build_s": round(pinfo["ch_seconds"], 2),
                      "builder": "GPU contraction (ch_gpu.cpp), identical to the host build"}
        if pinfo else None,
        # the whole step's real HBM traffic (PMC, every build kernel of the
        # child's one step, both streams) over the timed step
        "step_pmc": step_pmc(traffic, elapsed_max / args.steps),
        "pmc_traffic_per_launch": {k: {"launches": v["launches"],
                                       "bytes": round(v["bytes_per_launch"], 1),
                                       "read": round(v["read_bytes_per_launch"], 1),
                                       "write": round(v["write_bytes_per_launch"], 1)}
                                   for k, v in (traffic or {}).items()},
    }


BUILD_KERNELS = ("sweep_up", "sweep_down", "first_moves", "rle_count", "rle_fix", "rle_moves",
                 "rle_emit")


def step_pmc(traffic, step_s):
    """PMC bytes of one build step (the pmc child builds exactly one batch:
    every launch of every build kernel, on all streams) and the rate over the
    timed step."""
    if not traffic:
        return None
    b = sum(v["bytes_per_launch"] * v["launches"] for k, v in traffic.items() if k in BUILD_KERNELS)
    return {"GB": round(b / 1e9, 2), "TBps": round(b / step_s / 1e12, 3),
            "note": "2*FETCH_SIZE + WRITE_SIZE summed over the build kernels of one step / ms_per_step"}


# libcpd reports these counters through the timing table (launches = count)
_COUNTERS = ("wide_rows", "group_rows", "emit_sets", "pool_rebuilds")


# --------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the C oracle on host threads

def host_threads(args):
    """Every thread this job may use: OMP_NUM_THREADS when the box sets it
    (the GPU box's share is 16 of a much larger host), else the affinity."""
    if args.cpu_threads:
        return args.cpu_threads
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def host_info(threads):
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "threads": threads,
            "cpu_model": model, "omp_proc_bind": "unset (see _child_env)",
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS", "")}


def _child_env(threads):
    """A clean OpenMP environment for a CPU leg: its own process (torch's and
    libcpd's OpenMP runtimes in the bench process may have pinned the main
    thread), `threads` threads, no binding.  OMP_PROC_BIND=close was measured
    harmful here: the job's CPU share is a quota over all host CPUs (affinity
    = every CPU), so bound workers all start at CPU 0 and stack on the same
    cores (r02: the concurrent mod-3 run at a third of the sequential rate)."""
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    env.pop("OMP_PROC_BIND", None)
    env.pop("OMP_PLACES", None)
    return env


def cpu_worker(spec):
    """One timed CPU leg in a child process: CPD rows (reverse Dijkstra +
    first moves + RLE) for its targets, then table-search over them, with the
    C oracle on `threads`.  Targets: worker `wid` of `mod 3` (a sample of
    `rows`), or the list in `targets_npy`."""
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import cpd
    import oracle
    sp = json.loads(spec)
    g = cpd.synth_road_graph(sp["width"], sp["width"], seed=sp["seed"], style=sp["style"])
    order = oracle.dfs_preorder(g.row_ptr, g.dst)
    if sp.get("kind") == "search":
        cpu_search_leg(sp, g, order)
        return
    rng = np.random.default_rng(sp.get("qseed", 10 + sp.get("wid", 0)))
    if sp.get("targets_npy"):
        targets = np.load(sp["targets_npy"]).astype(np.uint32)
    else:
        mine = cpd.owned_nodes(g.n, 3, "mod", 3, sp["wid"])
        targets = np.sort(rng.choice(mine, sp["rows"], replace=False)).astype(np.uint32)
    s = rng.integers(0, g.n, sp["queries"]).astype(np.uint32)
    t = targets[rng.integers(0, len(targets), sp["queries"])]
    t0 = time.perf_counter()
    off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, targets, threads=sp["threads"])
    t1 = time.perf_counter()
    _, hops, _ = oracle.table_search(g.row_ptr, g.dst, g.w, order, targets, off, runs, s, t,
                                     threads=sp["threads"])
    t2 = time.perf_counter()
    print(json.dumps({"rows_s": t1 - t0, "queries_s": t2 - t1, "rows": len(targets),
                      "queries": len(s), "runs": int(off[-1]), "hops": int(hops.sum()),
                      "n": g.n, "m": g.m}), flush=True)


def cpu_search_leg(sp, g, order):
    """CPD-heuristic search on the host: the oracle's
    ora_cpd_search (the restated warthog cpd_search, OpenMP over queries) on
    the bench's 256 search rows and .diff stand-in weights, for each leg the
    first queries of the GPU's query list in chunks until a time budget is
    spent (so the default bench stays within minutes); q/s = queries done /
    their time."""
    import numpy as np
    import cpd
    import oracle
    srows = np.load(sp["targets_npy"]).astype(np.uint32)
    w_cong = cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3)
    off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, srows, threads=sp["threads"])
    out = {}
    for leg in sp["legs"]:
        q = np.load(leg["queries_npy"]).astype(np.uint32)
        s, t = q[0], q[1]
        done, secs, expanded = 0, 0.0, 0
        while done < leg["queries"] and secs < leg["budget_s"]:
            k = min(leg["chunk"], leg["queries"] - done)
            t0 = time.perf_counter()
            _, _, _, st = oracle.cpd_search(g.row_ptr, g.dst, g.w, w_cong, order, srows, off, runs,
                                            s[done:done + k], t[done:done + k],
                                            fscale=leg["fscale"], threads=sp["threads"])
            secs += time.perf_counter() - t0
            expanded += int(st[:, 0].sum())
            done += k
        out[leg["name"]] = {"queries": done, "s": secs, "queries_per_s": done / secs if secs else 0.0,
                            "mean_expanded": expanded / max(1, done)}
    print(json.dumps(out), flush=True)


def run_cpu_worker(spec, threads, timeout=900):
    p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker",
                          json.dumps(dict(spec, threads=threads))], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, env=_child_env(threads))
    return p


def collect(p, timeout=900):
    o, e = p.communicate(timeout=timeout)
    if p.returncode:
        raise RuntimeError(e[-400:])
    return json.loads(o.strip().splitlines()[-1])


def cpu_partitioned(threads, rows_per_worker=384, queries=20000):
    """configs[0] on the 300k stand-in (mod 3): three workers one after another
    with every thread, then all three at once with a third each."""
    spec = lambda wid: {"width": 548, "seed": 1, "style": "spec", "wid": wid,
                        "rows": rows_per_worker, "queries": queries}
    seq = [collect(run_cpu_worker(spec(wid), threads)) for wid in range(3)]
    per = max(1, threads // 3)
    procs = [run_cpu_worker(spec(wid), per) for wid in range(3)]
    con = [collect(p) for p in procs]
    rows = sum(r["rows"] for r in seq)
    q = sum(r["queries"] for r in seq)
    return {
        "graph": "melb stand-in: 548x548 spec-style synthetic (300,304 nodes), seed 1, mod 3",
        "rows_per_worker": rows_per_worker, "queries_per_worker": queries,
        "mean_runs_per_row": round(sum(r["runs"] for r in seq) / rows, 1),
        "sequential": {"threads_per_worker": threads,
                       "rows_per_s": round(rows / sum(r["rows_s"] for r in seq), 2),
                       "queries_per_s": round(q / sum(r["queries_s"] for r in seq), 1)},
        "concurrent": {"threads_per_worker": per,
                       "rows_per_s": round(rows / max(r["rows_s"] for r in con), 2),
                       "queries_per_s": round(q / max(r["queries_s"] for r in con), 1)},
    }


# --------------------------------------------------------------------------
# end-to-end worker build: bin/make_cpd_auto
# as the driver runs it (make_cpds.py:20), on a cold plan cache, every row the
# rank owns built, copied out of HBM and written to its bucket files in the
# compact layout (DOSCPD03: a 1/2/4-bit move per column by max out-degree,
# striped over part files); then
# bin/fifo_auto (make_fifos.py:21) loads those files and answers a request
# through the reference's FIFO protocol, checked against the oracle

def full_build_xy(args):
    """The workload's graph as a .xy file (bin/gen_synth, same generator and
    seed), written once per cache."""
    prefix = glob_xy(args)[:-3]
    if not os.path.exists(prefix + ".xy"):
        subprocess.run([os.path.join(ROOT, "bin", "gen_synth"), "--width", str(args.width),
                        "--seed", str(args.seed), "--style", args.style, "--out", prefix],
                       check=True, stdout=subprocess.DEVNULL, timeout=300)
    return prefix + ".xy"


def full_build_workers(args, world):
    """Workers of the configuration's partition the full-build leg runs: the
    partition key's (div 8: 8 workers, configs[3]'s "div 8"), or the rank
    count if larger.  Rank r runs worker r, so every rank builds one whole
    worker at any N (weak scaling, like the steps)."""
    return max(world, args.partkey)


def full_build_dir(args, world):
    return os.path.join(args.cache, f"fb-out-{world}")


def full_build(args, xy, world, rank, device, comm, runner=subprocess.run):
    """Run make_cpd_auto for worker `rank` of full_build_workers() with a
    fresh (cold) plan cache shared by the node's ranks; returns its JSON phase
    line.  Rank 0 writes its bucket files (DOSCPD03) into the cache directory
    on the box's disk; the other ranks run the same worker path with
    --discard (D2H export, no file writes): eight 31-GB workers would
    outgrow one node's disk."""
    import glob
    import shutil
    outdir = full_build_dir(args, world)
    if rank == 0:  # the previous runs' outputs (and plan caches) go first
        for d in glob.glob(os.path.join(args.cache, "fb-out-*")):
            shutil.rmtree(d, ignore_errors=True)
        os.makedirs(outdir)
    # no rank starts before the cold directory exists (a rank
    # that only polled for the directory could reuse a stale plan cache or
    # race rank 0's removal)
    comm.barrier()
    write = rank == 0 and not args.full_build_discard
    cmd = [os.path.join(ROOT, "bin", "make_cpd_auto"), "--input", xy, "--partmethod",
           args.partmethod, "--partkey", str(args.partkey), "--workerid", str(rank),
           "--maxworker", str(full_build_workers(args, world)), "--outdir", outdir, "--device",
           str(device), "--format", "moves"] + ([] if write else ["--discard"])
    if args.batch:
        cmd += ["--batch", str(args.batch)]
    p = runner(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=900)
    if p.returncode:
        raise RuntimeError(f"make_cpd_auto failed: {p.stderr[-400:]}")
    line = next(l for l in p.stdout.splitlines() if l.startswith("make_cpd_auto-json: "))
    rec = json.loads(line.split(": ", 1)[1])
    if write:
        rec["files_bytes"] = sum(os.path.getsize(os.path.join(outdir, f))  # with the part files
                                 for f in os.listdir(outdir) if ".cpd" in f and not f.endswith(".tmp"))
    return rec


def full_build_leg(args, xy, world, rank, device, comm, runner=subprocess.run):
    """full_build() on every rank, then the node's figures: the slowest
    worker's time, rows / runs / exported bytes summed over ranks (rank 0's
    phase record kept whole)."""
    rec = full_build(args, xy, world, rank, device, comm, runner)
    (tmax,) = comm.reduce([rec["total_s"]], "MAX")
    tot = comm.reduce([float(rec["rows"]), float(rec["runs"]), float(rec["export_bytes"])], "SUM")
    # every worker's own figures: which one limits the node
    allr = comm.gather([float(rec["worker"]), rec["total_s"], float(rec["rows"]),
                        float(rec.get("rows_s", 0.0))])
    W = full_build_workers(args, world)
    fb = {"what": f"bin/make_cpd_auto worker(s) 0..{world - 1} of {W} ({args.partmethod} "
                  f"{args.partkey}), one worker per rank: all its rows, cold plan cache, "
                  "compact bucket files (DOSCPD03, striped) written by rank 0, --discard (D2H export "
                  "only) on the other ranks",
          "total_s": round(tmax, 3), "rows": int(tot[0]), "runs": int(tot[1]),
          "rows_per_s_end_to_end": round(tot[0] / tmax, 1) if tmax else 0.0,
          "export_GB": round(tot[2] / 1e9, 2),
          "rank0": rec,
          "rank0_export_GBps": round(rec["export_bytes"] / rec["export_span_s"] / 1e9, 2)
          if rec.get("export_span_s") else None,
          "per_rank": [{"rank": r, "worker": int(v[0]), "total_s": round(v[1], 3), "rows": int(v[2]),
                        "rows_per_s": round(v[2] / v[1], 1) if v[1] else 0.0,
                        "rows_phase_s": round(v[3], 3)} for r, v in enumerate(allr)],
          "slowest_rank": max(range(len(allr)), key=lambda r: allr[r][1]),
          "imbalance_max_over_min": round(max(v[1] for v in allr) / min(v[1] for v in allr), 4)
          if min(v[1] for v in allr) > 0 else None}
    if "files_bytes" in rec:
        fb["files_GB"] = round(rec["files_bytes"] / 1e9, 2)
    return fb, rec


def _read_ready(p, deadline):
    """fifo_auto's load record and its "listening" line (raw reads of the
    pipe after select, with a deadline: a server that never comes up fails
    the leg, not the bench)."""
    import select
    fd = p.stdout.fileno()
    buf = b""
    while time.time() < deadline:
        r, _, _ = select.select([fd], [], [], 1.0)
        if r:
            chunk = os.read(fd, 65536)
            if not chunk:
                break
            buf += chunk
            if b"listening" in buf:
                rec = None
                for line in buf.decode(errors="replace").splitlines():
                    if line.startswith("fifo_auto-json: "):
                        rec = json.loads(line.split(": ", 1)[1])
                return rec
        if p.poll() is not None:
            break
    p.kill()
    raise RuntimeError(f"fifo_auto did not come up: {buf.decode(errors='replace')[-300:]} "
                       f"{p.stderr.read()[-300:]}")


CONF_DEFAULT = {"hscale": 1.0, "fscale": 0.0, "time": 0, "itrs": -1, "k_moves": -1, "threads": 0,
                "verbose": False, "debug": False, "thread_alloc": False, "no_cache": False}


def _serve_start(args, xy, outdir, W, device, alg, fifo):
    """bin/fifo_auto as make_fifos.py:21 starts it (resident; its FIFO at
    `fifo`): (process, its load record, seconds until it listens)."""
    cmd = [os.path.join(ROOT, "bin", "fifo_auto"), "--input", xy, xy + ".diff", "--partmethod",
           args.partmethod, "--partkey", str(args.partkey), "--workerid", "0", "--maxworker",
           str(W), "--outdir", outdir, "--alg", alg, "--device", str(device), "--fifo", fifo,
           "--verbose"]
    t0 = time.time()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    rec = _read_ready(p, t0 + 300)
    return p, rec, time.time() - t0


def _write_queries(path, s, t):
    """The query file process_query.send_queries writes (process_query.py:
    93-96): "{n}\n" then "s t" lines."""
    import numpy as np
    body = np.char.add(np.char.add(s.astype(str), " "), t.astype(str))
    with open(path, "w") as f:
        f.write(f"{len(s)}\n")
        if len(s):
            f.write("\n".join(body.tolist()) + "\n")


def _serve_request(fifo, outdir, name, s, t, diff="-", **conf):
    """One request through the reference's protocol (process_query.py:66-111:
    query file on the shared directory, answer FIFO made first, the JSON
    config + "qfile answer diff" line written to the worker's FIFO, the one
    stats line read back).  Returns (stats line, wall seconds from writing
    the request to reading the answer, query file)."""
    qfile = os.path.join(outdir, f"query.{name}")
    _write_queries(qfile, s, t)
    answer = os.path.join(outdir, f"answer.{name}")
    if os.path.exists(answer):
        os.remove(answer)
    os.mkfifo(answer)
    t1 = time.time()
    with open(fifo, "w") as f:  # process_query.py:89
        f.write(json.dumps(dict(CONF_DEFAULT, **conf)) + "\n" + f"{qfile} {answer} {diff}\n")
    with open(answer) as f:
        line = f.read().strip()
    wall = time.time() - t1
    os.remove(answer)
    return line, wall, qfile


def _serve_stop(p, fifo):
    """Ends the server ("quit"); returns its per-request phase records
    (--verbose: read + parse, prepare, compute seconds)."""
    try:
        with open(fifo, "w") as f:
            f.write("quit\n")
        p.wait(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    err = p.stderr.read().decode(errors="replace") if p.stderr else ""
    return [json.loads(ln.split(": ", 1)[1]) for ln in err.splitlines()
            if ln.startswith("fifo_auto-req: ")]


def _stats(line):
    """The worker's 10-field line (process_query.py:199-208), times in s."""
    v = [int(x) for x in line.split(",")]
    return {"n_expanded": v[0], "n_inserted": v[1], "n_touched": v[2], "n_updated": v[3],
            "n_surplus": v[4], "plen": v[5], "finished": v[6], "t_receive_s": v[7] / 1e9,
            "t_astar_s": v[8] / 1e9, "t_search_s": v[9] / 1e9}


def serve_leg(args, xy, outdir, W, device, g, order, threads, nprobe=4, big=1_000_000,
              probe_q=4000, search_q=65536, search_probe_q=1000):
    """The drop-in server on the bucket files worker 0 just wrote (VERDICT
    r04 item 1): bin/fifo_auto --alg table-search (make_fifos.py:21) with a
    probe request (debug side file, `nprobe` of the worker's targets) checked
    against the oracle, then one timed request of `big` queries (s uniform, t
    uniform over all the worker's targets; debug off) — q/s through the
    protocol and the worker's own t_receive / t_search split; then bin/
    fifo_auto --alg cpd-search on the same files, congested weights (the
    .diff gen_synth wrote beside the .xy), fscale 0.1: a probe request checked
    against the oracle's ora_cpd_search and a timed request of `search_q`."""
    import numpy as np
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpd
    import oracle
    rng = np.random.default_rng(7)
    mine = cpd.owned_nodes(g.n, W, args.partmethod, args.partkey, 0)
    probes = np.sort(rng.choice(mine, nprobe, replace=False)).astype(np.uint32)
    off, runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, probes, threads=threads)
    out = {"what": "bin/fifo_auto on worker 0's bucket files through the reference FIFO protocol "
                   "(query file, answer FIFO, JSON config line): probe requests vs the oracle, "
                   "timed requests with debug off"}
    fifo = os.path.join(outdir, "worker0.fifo")
    # ---- table-search
    p, rec, ready = _serve_start(args, xy, outdir, W, device, "table-search", fifo)
    try:
        s = rng.integers(0, g.n, probe_q).astype(np.uint32)
        t = probes[rng.integers(0, nprobe, probe_q)]
        line, wall, qfile = _serve_request(fifo, outdir, "probe", s, t, debug=True)
        res = np.loadtxt(qfile + ".res", dtype=np.uint64, ndmin=2)
        rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, order, probes, off, runs, s, t,
                                         threads=threads)
        exact = bool(len(res) == probe_q and np.array_equal(res[:, 0], s)
                     and np.array_equal(res[:, 2], rc) and np.array_equal(res[:, 3], rh)
                     and np.array_equal(res[:, 4], rf))
        bs = rng.integers(0, g.n, big).astype(np.uint32)
        bt = mine[rng.integers(0, len(mine), big)].astype(np.uint32)
        _serve_request(fifo, outdir, "warm", bs, bt)  # first request of this size: buffers
        bline, bwall, _ = _serve_request(fifo, outdir, "big", bs, bt)
    finally:
        reqs = _serve_stop(p, fifo)
    st = _stats(bline)
    out.update({"ready_s": round(ready, 3), "load": rec, "probe_queries": probe_q,
                "probe_targets": nprobe, "answer": line, "bit_exact": exact,
                "request_s": round(wall, 3),
                "table_search": {"queries": big, "wall_s": round(bwall, 4),
                                 "queries_per_s": round(big / bwall, 1),
                                 "t_receive_s": st["t_receive_s"], "t_search_s": st["t_search_s"],
                                 "finished": st["finished"], "answer": bline,
                                 "phases": reqs[-1] if reqs else None,
                                 "note": "wall = request written to answer read (the head's "
                                         "t_partition without ssh); the query file is written "
                                         "before, as process_query's t_prepare"}})
    # ---- cpd-search (walks form: the worker's 125k rows have no room for
    # per-row tables), congested weights, fscale 0.1
    w_cong = cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3)  # == gen_synth's .diff
    p, rec2, ready2 = _serve_start(args, xy, outdir, W, device, "cpd-search", fifo)
    try:
        s = rng.integers(0, g.n, search_probe_q).astype(np.uint32)
        t = probes[rng.integers(0, nprobe, search_probe_q)]
        line2, _, qfile = _serve_request(fifo, outdir, "sprobe", s, t, diff=xy + ".diff",
                                         fscale=0.1, debug=True)
        res = np.loadtxt(qfile + ".res", dtype=np.uint64, ndmin=2)
        rc, rp, rf, _ = oracle.cpd_search(g.row_ptr, g.dst, g.w, w_cong, order, probes, off, runs,
                                          s, t, fscale=0.1, threads=threads)
        sexact = bool(len(res) == search_probe_q and np.array_equal(res[:, 2], rc)
                      and np.array_equal(res[:, 3], rp) and np.array_equal(res[:, 4], rf))
        ss = rng.integers(0, g.n, search_q).astype(np.uint32)
        stt = mine[rng.integers(0, len(mine), search_q)].astype(np.uint32)
        sline, swall, _ = _serve_request(fifo, outdir, "sbig", ss, stt, diff=xy + ".diff",
                                         fscale=0.1)
    finally:
        sreqs = _serve_stop(p, fifo)
    st2 = _stats(sline)
    out["cpd_search"] = {"ready_s": round(ready2, 3), "probe_queries": search_probe_q,
                         "probe_answer": line2, "bit_exact": sexact, "fscale": 0.1,
                         "queries": search_q, "wall_s": round(swall, 4),
                         "queries_per_s": round(search_q / swall, 1),
                         "t_receive_s": st2["t_receive_s"], "t_astar_s": st2["t_astar_s"],
                         "t_search_s": st2["t_search_s"],
                         "queries_per_s_search": round(search_q / st2["t_search_s"], 1)
                         if st2["t_search_s"] else None,
                         # t_search = the passes + the per-row tables (round 5
                         # on; t_receive excluded), t_astar = the passes only
                         # (ADVICE r05): the receive-inclusive rate compares
                         # with round-4 records
                         "queries_per_s_receive_and_search":
                             round(search_q / (st2["t_receive_s"] + st2["t_search_s"]), 1)
                             if st2["t_search_s"] else None,
                         "t_search_definition": "t_search = search passes + per-row tables "
                                                "(t_receive not included); t_astar = passes",
                         "finished": st2["finished"], "mean_expanded": round(st2["n_expanded"] / search_q, 1),
                         "answer": sline, "phases": sreqs[-1] if sreqs else None}
    return out


def build_plan_child(args, ppath, device):
    """The workload's plan, its hierarchy contracted on GPU `device`
    (ch_gpu.cpp: the host build's hierarchy, arc for arc), in a child process
    so that this one initialises the GPU only after the PMC children."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import cpd\n"
            "g = cpd.synth_road_graph(%d, %d, seed=%d, style=%r)\n"
            "cpd.Plan(g, gpu=%d).save(%r)\n"
            % (PKG, args.width, args.width, args.seed, args.style, device, ppath))
    subprocess.run([sys.executable, "-c", code], check=True, timeout=600)


def glob_xy(args):
    style = "" if args.style == "shuffled" else f"-{args.style}"
    return os.path.join(args.cache, f"fb-synth{args.width}-s{args.seed}{style}.xy")


def full_build_only(args, world, rank, local):
    """The end-to-end worker leg alone (--full-build-only): rank r runs
    make_cpd_auto for worker r, rank 0 writes its files and serves them, the
    ranks' figures are gathered through files (FileComm) — these processes
    load neither torch nor HIP until every worker is done, so an 8-rank
    rehearsal on one GPU (CPD_BENCH_SHARE_GPU=1) holds the 8 workers and the
    launcher, within the box's 16 GPU processes.  One JSON line on rank 0."""
    share = os.environ.get("CPD_BENCH_SHARE_GPU") == "1"
    gpu = 0 if share else local
    if share and args.batch == 0:  # eight workers' batch buffers on one card
        args.batch = 1024
    os.makedirs(args.cache, exist_ok=True)
    # a directory per launch (the launcher's run id and port) for FileComm
    run_id = f"{os.environ.get('TORCHELASTIC_RUN_ID', 'solo')}-{os.environ.get('MASTER_PORT', '0')}"
    comm = FileComm(world, rank, local, os.path.join(args.cache, f"fb-comm-{world}-{run_id}"))
    xy = full_build_xy(args) if local == 0 else None
    comm.barrier()
    xy = xy or glob_xy(args)
    t0 = time.time()
    fb, rec = full_build_leg(args, xy, world, rank, gpu, comm)
    W = full_build_workers(args, world)
    if rank == 0 and "files_bytes" in rec:  # every worker is done: rank 0 alone on the GPU
        sys.path.insert(0, PKG)
        import cpd
        g = cpd.synth_road_graph(args.width, args.width, seed=args.seed, style=args.style)
        try:
            fb["serve"] = serve_leg(args, xy, full_build_dir(args, world), W, gpu, g,
                                    cpd.dfs_preorder(g.row_ptr, g.dst), host_threads(args))
        except Exception as e:  # reported
            fb["serve"] = {"error": str(e)[-400:]}
    comm.barrier()
    if rank == 0:
        import shutil
        shutil.rmtree(full_build_dir(args, world), ignore_errors=True)
        print(json.dumps({"what": "full-build leg only", "n_gpus": world,
                          "shared_gpu_rehearsal": share, "batch": args.batch or "auto",
                          "wall_s": round(time.time() - t0, 3), "full_build": fb}), flush=True)


def main():
    args = parse()
    if args.cpu_worker:
        cpu_worker(args.cpu_worker)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world == 1:
        # not under torch.distributed.run: launch ourselves that way (a child,
        # before anything touches the GPU)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
               "--master-port", os.environ.get("MASTER_PORT", "29517"), __file__] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if args.pmc_child:
        pmc_child(args)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.full_build_only:
        full_build_only(args, world, rank, local)
        return

    import numpy as np
    import torch  # first: libcpd then binds to the same HIP runtime
    import torch.distributed as dist

    sys.path.insert(0, PKG)
    import cpd

    # ---- graph + host preprocessing (cached, built once per node; host only)
    t0 = time.time()
    g = cpd.synth_road_graph(args.width, args.width, seed=args.seed, style=args.style)
    os.makedirs(args.cache, exist_ok=True)
    ppath = plan_path(args)
    if local == 0 and not os.path.exists(ppath):
        log(f"building hierarchy for {g.n} nodes / {g.m} edges on GPU {local} ...")
        build_plan_child(args, ppath, local)
    fb_xy = None
    if not args.no_full_build and args.sample is None and local == 0:
        fb_xy = full_build_xy(args)
    # PMC passes: children, before this process initialises the GPU.  At N > 1
    # on rank 0 only, on its own GPU (device 0 = local rank 0's), while the
    # other ranks wait in the process group's rendezvous: every rank builds
    # the same shape of batch, so rank 0's bytes per launch stand for all
    # (an N > 1 roofline says where its traffic is from)
    # CPD_BENCH_SHARE_GPU=1 (rehearsal on a 1-GPU box only): every rank uses
    # GPU 0 and the harness collectives go over gloo.  Never used for numbers.
    share = os.environ.get("CPD_BENCH_SHARE_GPU") == "1"
    gpu = 0 if share else local
    if share and args.batch == 0:  # ranks sized from one card's free HBM would overcommit it
        args.batch = 4096
    # the search workspaces' share of free HBM: ranks sharing one card split it
    # (the library's default share per rank would overcommit it)
    wf = 0.6 / world if share else 0.0
    traffic = None
    if rank == 0 and local == 0 and not args.no_pmc:
        traffic = pmc_traffic(args)
    # CPD_BENCH_PG=1: the process group (RCCL) even at one rank, so the N>1
    # collectives' code path runs on a 1-GPU box too
    use_pg = world > 1 or os.environ.get("CPD_BENCH_PG") == "1"
    if use_pg and not share:
        global _RESULT_FD
        sys.stdout.flush()
        _RESULT_FD = os.dup(1)
        os.dup2(2, 1)
    if use_pg:
        if share:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    comm = Comm(world, rank, local, device=None if share else f"cuda:{local}", pg=use_pg)
    comm.barrier()
    while not os.path.exists(ppath):  # another local rank is still saving it
        time.sleep(0.5)
    plan = cpd.Plan.load(ppath)
    pinfo = plan.info()
    assert pinfo["n"] == g.n and pinfo["m"] == g.m
    log(f"rank {rank}: plan ready in {time.time() - t0:.1f}s (hierarchy build "
        f"{pinfo['ch_seconds']:.1f}s, {pinfo['ch_up_arcs'] + pinfo['ch_dn_arcs']} arcs, levels "
        f"{pinfo['levels_up']}+{pinfo['levels_dn']})")

    dev = cpd.Graph(plan, device=gpu, batch=args.batch)
    # batch lanes along a Hilbert curve of the node coordinates (compact
    # 256-target groups: narrow rows fit; identical rows either way)
    dev.set_coords(g.x, g.y)
    # every rank builds the same number of rows per step (weak scaling): the
    # smallest batch any rank's free HBM allows
    (bmin,) = comm.reduce([float(dev.batch)], "MIN")
    if int(bmin) != dev.batch:
        dev.set_batch(int(bmin))
    B = dev.batch
    owned = rank_targets(args, g.n, world, rank)
    if len(owned) == 0:
        raise SystemExit(f"rank {rank} owns no targets")

    rows = None
    for i in range(args.warmup):
        rows = dev.build_rows(batch_of(owned, B, i), reuse=rows)
    dev.timing(not args.no_timing)
    dev.timing_reset()
    comm.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        # step i + 1's targets: its up-sweep starts beside step i's first
        # moves (cpd_graph_hint_next); none across the timed region's edges,
        # so the region holds exactly `steps` batches of every kernel
        if i + 1 < args.steps:
            dev.hint_next(batch_of(owned, B, args.warmup + i + 1))
        rows = dev.build_rows(batch_of(owned, B, args.warmup + i), reuse=rows)
    rows.wait()  # the last batch's run emit, inside the timed region
    comm.barrier()
    elapsed = time.perf_counter() - t0
    (elapsed_max,) = comm.reduce([elapsed], "MAX")
    ranks = rank_table(B, args.steps, [v[0] for v in comm.gather([elapsed])])
    kt = dev.timing_get()
    dev.timing(False)
    nrows, nruns = rows.count()
    last_targets = batch_of(owned, B, args.warmup + args.steps - 1)

    # ---- table-search ------------------------------------------------------
    rng = np.random.default_rng(100 + rank)
    extra = {}
    w_cong = cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3)
    runs_form = None
    if args.sample is None:
        # the rank's last batch of rows, kept as RLE too (both forms timed).
        # Making this index decodes the batch's run words into HBM
        # (moves_runs): the reference's own row form (warthog's RLE words,
        # README.md:92-93), timed here so the line states its cost (VERDICT
        # r04 item 8)
        dev.timing(True)
        dev.timing_reset()
        ix = cpd.Index(dev, rows=rows)
        dkt = dev.timing_get()
        dev.timing(False)
        dec = dkt.get("moves_runs")
        if dec and dec["ms"] > 0:
            step_s = elapsed_max / args.steps
            runs_form = {"decode_ms_per_batch": round(dec["ms"], 3),
                         "decode_GBps": round(dec["bytes"] / (dec["ms"] / 1e3) / 1e9, 1),
                         "rows_per_s_runs": round(world * B / (step_s + dec["ms"] / 1e3), 1),
                         "note": "a step that also decodes its batch's run words into HBM "
                                 "(moves_runs after the build, not overlapped)"}
        nq = args.queries
        qs = rng.integers(0, g.n, nq).astype(np.uint32)
        qt = last_targets[rng.integers(0, len(last_targets), nq)]
        index_rows = len(last_targets)
    else:
        # every row the worker owns, streamed batch by batch into dense tables
        ti = time.perf_counter()
        ix = cpd.Index.streamed(dev, owned, 1 << 62, mode="dense")
        for a in range(0, len(owned), B):
            rows = dev.build_rows(owned[a:a + B], reuse=rows)
            ix.append_rows(rows)
        comm.barrier()
        extra["worker_index_build_s"] = round(time.perf_counter() - ti, 3)
        del rows
        rows = None
        index_rows = len(owned)
        # the 10M-query batch: t uniform over the sample (seed 6), s uniform;
        # this worker's share is what the head routes to it
        qrng = np.random.default_rng(6)
        allt = sample_nodes(g.n, *args.sample)[qrng.integers(0, args.sample[0], args.queries)]
        alls = qrng.integers(0, g.n, args.queries).astype(np.uint32)
        mine = np.isin(allt, owned)
        qs, qt = alls[mine], allt[mine]
        nq = len(qs)
        extra["worker_queries"] = nq
    ix.prepare(qs, qt)

    def time_queries(mode, reps=3):
        ix.set_mode(mode)
        ix.run()  # warm (and, for dense, expand the rows once)
        ms, hops = 0.0, 0
        for _ in range(reps):
            st = ix.run()
            ms += st["kernel_ms"]
            hops += st["hops"]
        tot = comm.reduce([float(nq * reps), ms, float(hops)], "SUM")
        (ms_max,) = comm.reduce([ms], "MAX")
        return tot, ms_max

    q_rle = q_rle_ms = None
    if args.sample is None:
        q_rle, q_rle_ms = time_queries("rle")
    q_totals, q_ms_max = time_queries("auto")
    index_mode = ix.mode
    # end to end: host arrays in, host arrays out —
    # cpd_query_batch = prepare (upload, target sort on the GPU) + walk +
    # fetch (results back in caller order), by the host clock
    ix.query(qs, qt)  # warm
    te = time.perf_counter()
    for _ in range(3):
        ix.query(qs, qt)
    e2e_s = time.perf_counter() - te
    (e2e_max,) = comm.reduce([e2e_s], "MAX")
    (e2e_q,) = comm.reduce([float(3 * nq)], "SUM")
    ix.prepare(qs, qt)
    # congested leg (configs[2]): the .diff stand-in of SURVEY.md §8d — 10% of
    # edges x U[1, 3], rounded up — sent with the batch as fifo_auto does
    ix.set_weights(w_cong)
    q_cong, q_cong_ms = time_queries("auto")
    ix.set_weights(None)
    del ix, rows
    # The build's batch buffers (~190 GB at 1M nodes) are not used past this
    # point: the search, CPU-baseline and parity legs run on a graph with
    # 1024-row batches, which leaves the HBM to the search workspaces.
    import gc
    del dev
    gc.collect()
    dev = cpd.Graph(plan, device=gpu, batch=1024)
    dev.set_coords(g.x, g.y)
    # CPD-heuristic search leg: 256 rows of the index, the
    # .diff stand-in weights, hscale 1 / fscale 0.1 (10%-bounded: at fscale 0
    # a 1M-node search inserts up to ~235k nodes, a lane-serial search's
    # worst case), 65536 queries (20k in round 3-4: 329k q/s; 65536 fill the
    # 1024 search waves: 820k, profiles/r04ar_bench_sq64k.json)
    search = None
    if args.sample is None and not args.no_search:
        log(f"rank {rank}: cpd-search legs")
        srows = last_targets[:256]
        sr = dev.build_rows(srows)
        six = cpd.Index.streamed(dev, srows, sr.count()[1], mode="dense")
        six.append_rows(sr)
        del sr
        six.set_weights(w_cong)
        # every leg runs the library's workspace policy (capacity 0: the
        # first pass's columns per lane, the passes at 4x that resume the
        # searches that outgrew it, the share of HBM) — what fifo_auto runs
        sq = 65536  # as many searches as the 1024 search waves have lanes
        ss = rng.integers(0, g.n, sq).astype(np.uint32)
        st_ = srows[rng.integers(0, len(srows), sq)]
        wst = six.search(ss[:256], st_[:256], fscale=0.1, workspace_frac=wf)[4]  # warm: tables built here
        _, _, sfin, scnt, sst = six.search(ss, st_, fscale=0.1, workspace_frac=wf)
        tot = comm.reduce([float(sq), sst["kernel_ms"]], "SUM")
        (smax,) = comm.reduce([sst["kernel_ms"]], "MAX")

        def passes(stt):
            return {"capacity": int(stt["capacity"]), "capacity_last": int(stt["capacity_last"]),
                    "passes": int(stt["passes"]), "reruns": int(stt["reruns"]),
                    "resumed": int(stt["resumed"]), "restarted": int(stt["restarted"]),
                    "wasted_expanded": int(stt["wasted_expanded"])}
        # the headline is the memoised-walk form: what a
        # worker-sized index runs (fifo_auto; per-row tables of a div-8
        # worker's 125k rows would need 2.5 PB); the per-row tables form,
        # which only a small index holds, is reported beside it
        tables_form = {"queries_per_s": round(tot[0] / (smax / 1e3), 1) if smax else 0.0,
                       "queries": sq, "mean_expanded": round(float(scnt[:, 0].mean()), 1),
                       "finished": int(sfin.sum()), "overflow": int(sst["overflow"]),
                       "kernel_ms": round(sst["kernel_ms"], 3), "lanes": int(sst["lanes"]),
                       **passes(sst),
                       "form": {1: "per-row tables", 2: "memoised walks"}[sst["tables"]],
                       "tables_ms_per_row": round(wst["tables_ms"] / len(srows), 3)}
        # fscale 0 (optimal under the .diff weights): a 1M-node search expands
        # ~49k nodes; 65536 searches start at once in 2^15-column workspaces
        # and the ~60% that outgrow them spill their state and resume at 2^17
        # (then 2^19): each search is a latency chain, so lanes buy throughput
        # (profiles/search_lanes_ab/).  Ranks sharing one card in a rehearsal
        # split its HBM.
        # the fscale-0.1 queries with the memoised-walk form: the headline
        _, _, wfin, wcnt, wsst = six.search(ss, st_, fscale=0.1, tables="walks", workspace_frac=wf)
        wtot = comm.reduce([float(sq)], "SUM")
        (wmax,) = comm.reduce([wsst["kernel_ms"]], "MAX")
        search = {"queries_per_s": round(wtot[0] / (wmax / 1e3), 1) if wmax else 0.0,
                  "form": "memoised walks (what a worker-sized index runs)",
                  "config": "256-row dense index, .diff stand-in weights, hscale 1, fscale 0.1, "
                            "library workspace policy",
                  "queries": sq, "mean_expanded": round(float(wcnt[:, 0].mean()), 1),
                  "finished": int(wfin.sum()), "overflow": int(wsst["overflow"]),
                  "kernel_ms": round(wsst["kernel_ms"], 3), "lanes": int(wsst["lanes"]),
                  **passes(wsst), "tables_form": tables_form}
        zq = 65536
        zs = rng.integers(0, g.n, zq).astype(np.uint32)
        zt = srows[rng.integers(0, len(srows), zq)]
        six.search(zs[:64], zt[:64], workspace_frac=wf)  # warm
        _, _, zfin, zcnt, zst = six.search(zs, zt, workspace_frac=wf)
        ztot = comm.reduce([float(zq), zst["kernel_ms"]], "SUM")
        (zmax,) = comm.reduce([zst["kernel_ms"]], "MAX")
        search["fscale0"] = {
            "queries_per_s": round(ztot[0] / (zmax / 1e3), 1) if zmax else 0.0,
            "form": {1: "per-row tables", 2: "memoised walks"}[zst["tables"]],
            "queries": zq, **passes(zst), "lanes": int(zst["lanes"]),
            "mean_expanded": round(float(zcnt[:, 0].mean()), 1),
            "finished": int(zfin.sum()), "overflow": int(zst["overflow"]),
            "kernel_ms": round(zst["kernel_ms"], 3),
            # per-lane latency: one search's expansions in series
            "us_per_expansion_per_lane": round(zst["kernel_ms"] * 1e3 * int(zst["lanes"]) /
                                               max(1.0, float(zcnt[:, 0].sum())), 2)}

        search_sample = (six, ss[:2000], st_[:2000], srows, ss, st_, zs, zt)
    # walk kernel vs its roofline: per query 8 (s, t) + 4 (row) + 13 (cost,
    # moves, flag) bytes, per move the 4-B word holding the move + the 8-B edge
    qbytes = 25.0 * q_totals[0] + 12.0 * q_totals[2]
    qach = qbytes / (q_totals[1] / 1e3) / 1e9 if q_totals[1] else 0.0
    qkey = "table_search_dense" if index_mode == "dense" else "table_search"
    qt_pmc = (traffic or {}).get(qkey)
    query_roof = {"bound": "hbm", "kernel": qkey, "achieved": round(qach, 1),
                  "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(qach / HBM_PEAK_GBPS, 4),
                  "traffic": round(qt_pmc["bytes_per_launch"], 1) if qt_pmc else None,
                  "traffic_unit": "bytes/launch (PMC, 1M-query launch of the pmc child)",
                  "bytes_per_launch": round(qbytes / max(1, q_totals[0]) * nq, 1),
                  "avg_launch_ms": round(q_totals[1] / max(1.0, q_totals[0] / max(1, nq)), 3),
                  "note": "latency/request-bound dependent walk; HBM bytes are not its limit"}

    # ---- CPU baseline + full-size parity sample (rank 0, N = 1) -------------
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = host_threads(args)
        # ~10 s of CPU work: the per-row Dijkstra grows with n (64 rows per
        # thread at 1M nodes)
        per_thread = max(4, round(args.cpu_rows_per_thread * 1e6 / g.n))
        sample = batch_of(owned, B, 0)[: threads * per_thread]
        tnpy = os.path.join(args.cache, f"cpu-targets-{os.getpid()}.npy")
        np.save(tnpy, sample)
        cq = 20000
        leg = collect(run_cpu_worker({"width": args.width, "seed": args.seed, "style": args.style,
                                      "targets_npy": tnpy, "queries": cq, "qseed": 200},
                                     threads))
        os.remove(tnpy)
        # parity at full size (untimed): 128 of the sample's rows and 20k
        # queries over them, free-flow and congested, GPU against the oracle
        order = plan.order()
        psamp = sample[:: max(1, len(sample) // 128)][:128]
        ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, psamp, threads=threads)
        grows = dev.build_rows(psamp)
        goff, gruns = grows.export()
        parity = bool(np.array_equal(goff, ref_off) and np.array_equal(gruns, ref_runs))
        cs = rng.integers(0, g.n, cq).astype(np.uint32)
        ct = psamp[rng.integers(0, len(psamp), cq)]
        gix = cpd.Index(dev, rows=grows)
        for w_sel in (g.w, w_cong):
            rc, rh, _ = oracle.table_search(g.row_ptr, g.dst, w_sel, order, psamp, ref_off,
                                            ref_runs, cs, ct, threads=threads)
            gix.set_weights(None if w_sel is g.w else w_sel)
            gc_, gh, _, _ = gix.query(cs, ct)
            parity = parity and bool(np.array_equal(gc_, rc) and np.array_equal(gh, rh))
        del gix, grows
        if search:
            six, ss2, st2, srows, ss_all, st_all, zs, zt = search_sample
            # the same searches on the host (child process, every job thread)
            snpy = os.path.join(args.cache, f"cpu-search-{os.getpid()}.npy")
            qnpy = [os.path.join(args.cache, f"cpu-search-q{i}-{os.getpid()}.npy") for i in (0, 1)]
            np.save(snpy, srows)
            try:
                spec_legs = []
                for i, (name, qs_, qt_, fs, chunk, budget) in enumerate(
                        (("fscale0.1", ss_all, st_all, 0.1, 500, 8.0),
                         ("fscale0", zs, zt, 0.0, 2 * threads, 12.0))):
                    np.save(qnpy[i], np.stack([qs_, qt_]))
                    spec_legs.append({"name": name, "fscale": fs, "queries": len(qs_),
                                      "chunk": chunk, "budget_s": budget, "queries_npy": qnpy[i]})
                r = collect(run_cpu_worker({"kind": "search", "width": args.width,
                                            "seed": args.seed, "style": args.style,
                                            "targets_npy": snpy, "legs": spec_legs}, threads))
                legs = [r["fscale0.1"], r["fscale0"]]
                gpu_q = (search["queries_per_s"], search["fscale0"]["queries_per_s"])
                # (the GPU's fscale-0.1 figure is the walks form; the oracle
                # walks its rows' runs the same way, memo included)
                search["cpu_baseline"] = {
                    "kind": "port", "cores": threads,
                    "what": "oracle ora_cpd_search (restated cpd_search, OpenMP over queries) in "
                            "a child process, the GPU legs' first queries until a time budget",
                    "fscale0.1": dict(legs[0], gpu_over_cpu=round(gpu_q[0] / legs[0]["queries_per_s"], 2)
                                      if legs[0]["queries_per_s"] else None),
                    "fscale0": dict(legs[1], gpu_over_cpu=round(gpu_q[1] / legs[1]["queries_per_s"], 2)
                                    if legs[1]["queries_per_s"] else None)}
            except Exception as e:  # reported, never fatal to the GPU numbers
                search["cpu_baseline"] = {"error": str(e)[-300:]}
            finally:
                for f in [snpy] + qnpy:
                    if os.path.exists(f):
                        os.remove(f)
            sref = oracle.build_rows(g.row_ptr, g.dst, g.w, order, srows, threads=threads)
            rc, rp, rf, rs = oracle.cpd_search(g.row_ptr, g.dst, g.w, w_cong, order, srows,
                                               sref[0], sref[1], ss2, st2, fscale=0.1,
                                               threads=threads)
            gcs, gps, gfs, gcnt, _ = six.search(ss2, st2, fscale=0.1, workspace_frac=wf)
            search["parity_2000_bit_exact"] = bool(
                np.array_equal(gcs, rc) and np.array_equal(gps, rp) and np.array_equal(gfs, rf)
                and np.array_equal(gcnt.astype(np.uint64), rs))
            parity = parity and search["parity_2000_bit_exact"]
            # fscale 0: 64 queries against the oracle
            rc, rp, rf, rs = oracle.cpd_search(g.row_ptr, g.dst, g.w, w_cong, order, srows,
                                               sref[0], sref[1], ss2[:64], st2[:64],
                                               threads=threads)
            gcs, gps, gfs, gcnt, _ = six.search(ss2[:64], st2[:64], workspace_frac=wf)
            search["fscale0"]["parity_64_bit_exact"] = bool(
                np.array_equal(gcs, rc) and np.array_equal(gps, rp) and np.array_equal(gfs, rf)
                and np.array_equal(gcnt.astype(np.uint64), rs))
            parity = parity and search["fscale0"]["parity_64_bit_exact"]
        cpu = {"value": round(leg["rows"] / leg["rows_s"], 3), "unit": "sources/s",
               "cores": threads, "kind": "port",
               "sample": f"{leg['rows']} CPD rows of the same graph and partition (reverse "
                         f"Dijkstra + first moves + RLE, C oracle, OpenMP {threads} threads in a "
                         f"child process, {leg['rows_s']:.1f}s); table-search {cq} queries over "
                         f"them in {leg['queries_s']:.2f}s",
               "queries_per_s": round(leg["queries"] / leg["queries_s"], 1),
               "queries_form": "RLE rows, get_move by binary search over each row's runs (the "
                               "oracle's walk) — the GPU's queries_per_s walks dense move "
                               "tables, queries_per_s_rle the same RLE rows",
               "host": host_info(threads)}
        if not args.no_cpu_partitioned:
            try:
                cpu["partitioned_configs0"] = cpu_partitioned(threads)
            except Exception as e:  # reported, never fatal to the GPU numbers
                cpu["partitioned_configs0"] = {"error": str(e)[-300:]}

    # ---- end-to-end worker build: frees this process's HBM first ------------
    fb = None
    if not args.no_full_build and args.sample is None:
        import gc
        search_sample = six = None  # noqa: F841
        del dev
        gc.collect()
        comm.barrier()
        fb_xy = fb_xy or glob_xy(args)  # local rank 0 wrote it before the first barrier
        fb, rec = full_build_leg(args, fb_xy, world, rank, gpu, comm)
        W = full_build_workers(args, world)
        if rank == 0 and "files_bytes" in rec:
            try:
                fb["serve"] = serve_leg(args, fb_xy, full_build_dir(args, world), W, gpu, g,
                                        plan.order(), host_threads(args))
            except Exception as e:  # reported, never fatal to the GPU numbers
                fb["serve"] = {"error": str(e)[-400:]}
        comm.barrier()
        if rank == 0:  # the box's disk: the worker's files go once checked
            import shutil
            shutil.rmtree(full_build_dir(args, world), ignore_errors=True)

    if rank == 0:
        out = assemble(args, world, (g.n, g.m), B, elapsed_max, q_totals, q_ms_max, nrows, nruns,
                       kt, cpu, parity, pinfo, traffic)
        out["lib_src_sha"] = cpd.lib_src_sha()
        out["tree_src_sha"] = cpd.src_sha(ROOT)
        out["full_build"] = fb
        out["full_build_s"] = fb["total_s"] if fb else None
        out["query_index"] = index_mode
        out["query_index_rows_per_gpu"] = index_rows
        out["query_roofline"] = query_roof
        out["cpd_search"] = search
        if q_rle_ms:
            out["queries_per_s_rle"] = round(q_rle[0] / (q_rle_ms / 1e3), 1)
        out["queries_per_s_congested"] = (round(q_cong[0] / (q_cong_ms / 1e3), 1)
                                          if q_cong_ms else 0.0)
        out["queries_per_s_e2e"] = round(e2e_q / e2e_max, 1) if e2e_max else 0.0
        out["queries_e2e_note"] = ("cpd_query_batch by the host clock: (s, t) upload, target sort "
                                   "and gather on the GPU, walk, results scattered back and "
                                   "copied out")
        out["ranks"] = ranks
        out["runs_form"] = runs_form
        out["rows_per_s_runs"] = runs_form["rows_per_s_runs"] if runs_form else None
        out.update(extra)
        emit_line(json.dumps(out))
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
