#!/usr/bin/env python3
"""bench.py — MI355X CPD build (sources/s, GTEPS) and table-search (queries/s).

Workload (BASELINE.json configs[3]; melb-both.xy is a missing blob, so the
1M-node synthetic road graph the north star names is the headline graph):
  synthetic grid-perturbed road graph, 1000 x 1000 lattice (1M nodes, 2.5M
  edges), seed 1; partition `div 8` over the ranks (distribution_controller
  semantics), one rank per GPU.  A step = one batch of `--batch` CPD rows built
  from the rank's own targets: two CH sweeps, first-move sets and the RLE rows,
  all resident in HBM (weak scaling: every rank builds the same number of rows
  per step; no collective on the data path).  After the timed steps each rank
  runs `--queries` table-search queries against its last batch of rows.

One JSON line on rank 0: value = rows/s over all ranks; roofline for the
dominant kernel from HIP events; cpu_baseline = the C oracle (OpenMP) on a
bounded sample of the same workload, rank 0 at N = 1 only.

  python bench.py [--gpus N] [--steps K] [--warmup W]
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
PLAN_TAG = "ch823"      # bump when the hierarchy builder changes (cache key)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1000, help="lattice side (nodes = width^2)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--partmethod", default="div")
    ap.add_argument("--partkey", type=int, default=8)
    ap.add_argument("--batch", type=int, default=0,
                    help="rows per step (multiple of 1024); 0 = what fits in HBM, <= 16384")
    ap.add_argument("--queries", type=int, default=1_000_000)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores)")
    ap.add_argument("--cpu-rows-per-thread", type=int, default=64,
                    help="CPU baseline sample: rows per host thread (~10 s of CPU work)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 --pmc passes that fill roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cache", default=os.environ.get("CPD_BENCH_CACHE", "/tmp/cpd-bench-cache"))
    return ap.parse_args(argv)


# rocprofv3 kernel names -> the library's timing names
KERNEL_NAMES = {"sweep_level<true": "sweep_up", "sweep_up_": "sweep_up",
                "sweep_level<false": "sweep_down", "sweep_down8": "sweep_down",
                "first_moves": "first_moves", "rle_scan<false": "rle_count",
                "rle_scan<true": "rle_emit", "table_search": "table_search"}


def pmc_traffic(args, plan_path):
    """HBM traffic per launch from rocprofv3 PMC counters.

    One child run per counter (MI355X_MICROARCH.md: FETCH_SIZE costs 3 and
    WRITE_SIZE 2 of the 4 TCC slots, so they cannot share a pass), each a
    one-step build of the same workload.  Both counters are in KiB; on gfx950
    FETCH_SIZE reports half the bytes of a 16-B/lane streaming read, so it is
    doubled (our kernels' loads are 16 B per lane); WRITE_SIZE is exact for
    16-B stores.  Started before this process touches the GPU.  Returns
    {name: {"launches", "FETCH_SIZE", "WRITE_SIZE", "bytes_per_launch"}} or None.
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
               "--warmup", "0", "--width", str(args.width), "--seed", str(args.seed),
               "--partmethod", args.partmethod, "--partkey", str(args.partkey),
               "--batch", str(args.batch), "--cache", args.cache]
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
            name = next((v for k, v in KERNEL_NAMES.items() if k in row["Kernel_Name"]), None)
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
    """One build step under the profiler (no torch: nothing else on the GPU)."""
    sys.path.insert(0, PKG)
    import cpd
    plan = cpd.Plan.load(os.path.join(args.cache, f"synth{args.width}-s{args.seed}-{PLAN_TAG}.plan"))
    n = plan.info()["n"]
    dev = cpd.Graph(plan, device=0, batch=args.batch)
    owned = shard_targets(n, 1, args.partmethod, args.partkey, 0)
    dev.build_rows(batch_of(owned, dev.batch, 0))


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# --------------------------------------------------------------------------
# distributed plumbing (importable; tests/test_bench_dist.py runs it on gloo)

class Comm:
    """Barrier / reductions over torch.distributed.  Only the bench harness
    uses them (timing and a handful of counters); nothing on the data path."""

    def __init__(self, world, rank, local, device=None):
        self.world, self.rank, self.local, self.device = world, rank, local, device

    def barrier(self):
        import torch
        if self.device is not None:
            torch.cuda.synchronize()
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def reduce(self, vals, op):
        if self.world == 1:
            return list(vals)
        import torch
        import torch.distributed as dist
        t = torch.tensor(vals, dtype=torch.float64, device=self.device or "cpu")
        dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
        return t.tolist()


def shard_targets(nodenum, world, method, key, rank):
    """The rank's targets: distribution_controller partition, worker = rank."""
    sys.path.insert(0, PKG)
    import cpd
    return cpd.owned_nodes(nodenum, world, method, key, rank)


def batch_of(owned, B, i):
    """Step i's targets: the next B of the rank's own, wrapping around."""
    import numpy as np
    idx = (np.arange(B, dtype=np.int64) + i * B) % len(owned)
    return owned[idx]


def assemble(args, world, graph_info, B, elapsed_max, q_totals, q_ms_max, nrows, nruns,
             kt, cpu, parity, pinfo, traffic=None):
    """Rank 0's JSON line.  value = rows built by ALL ranks / max rank time.
    roofline: the kernel with the most device time; achieved = its algorithmic
    bytes (SURVEY.md §8d model, counted per launch by libcpd) / its summed
    event time; traffic = PMC bytes per launch of the same kernel (or None)."""
    n, m = graph_info
    total_rows = world * args.steps * B
    value = total_rows / elapsed_max
    roof = None
    if kt:
        name, k = max(kt.items(), key=lambda kv: kv[1]["ms"])
        achieved = k["bytes"] / (k["ms"] / 1e3) / 1e9 if k["ms"] > 0 else 0.0
        t = (traffic or {}).get(name)
        roof = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": round(t["bytes_per_launch"], 1) if t else None,
                "traffic_unit": "bytes/launch (PMC: 2*FETCH_SIZE + WRITE_SIZE, KiB->B)",
                "launches": k["launches"],
                "avg_launch_us": round(k["ms"] * 1e3 / max(1, k["launches"]), 3),
                "bytes_per_launch": round(k["bytes"] / max(1, k["launches"]), 1)}
    qps = q_totals[0] / (q_ms_max / 1e3) if q_ms_max > 0 else 0.0
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
                   "graph": f"grid-perturbed {args.width}x{args.width} seed {args.seed}",
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
        "hierarchy": {"arcs": pinfo["ch_up_arcs"] + pinfo["ch_dn_arcs"],
                      "levels": [pinfo["levels_up"], pinfo["levels_dn"]],
                      "build_s": round(pinfo["ch_seconds"], 1)} if pinfo else None,
        "pmc_traffic_per_launch": {k: {"launches": v["launches"],
                                       "bytes": round(v["bytes_per_launch"], 1),
                                       "read": round(v["read_bytes_per_launch"], 1),
                                       "write": round(v["write_bytes_per_launch"], 1)}
                                   for k, v in (traffic or {}).items()},
    }


# libcpd reports these counters through the timing table (launches = count)
_COUNTERS = ("wide_rows", "group_rows")


# --------------------------------------------------------------------------

def main():
    args = parse()
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

    import numpy as np
    import torch  # first: libcpd then binds to the same HIP runtime
    import torch.distributed as dist

    sys.path.insert(0, PKG)
    import cpd

    # ---- graph + host preprocessing (cached, built once per node; host only)
    t0 = time.time()
    g = cpd.synth_road_graph(args.width, args.width, seed=args.seed)
    os.makedirs(args.cache, exist_ok=True)
    plan_path = os.path.join(args.cache, f"synth{args.width}-s{args.seed}-{PLAN_TAG}.plan")
    if local == 0 and not os.path.exists(plan_path):
        log(f"building hierarchy for {g.n} nodes / {g.m} edges ...")
        cpd.Plan(g).save(plan_path)
    # PMC passes: children, before this process initialises the GPU
    traffic = None
    if world == 1 and not args.no_pmc:
        traffic = pmc_traffic(args, plan_path)

    # CPD_BENCH_SHARE_GPU=1 (rehearsal on a 1-GPU box only): every rank uses
    # GPU 0 and the harness collectives go over gloo.  Never used for numbers.
    share = os.environ.get("CPD_BENCH_SHARE_GPU") == "1"
    gpu = 0 if share else local
    if share and args.batch == 0:  # ranks sized from one card's free HBM would overcommit it
        args.batch = 4096
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    comm = Comm(world, rank, local, device=None if share else f"cuda:{local}")
    comm.barrier()
    plan = cpd.Plan.load(plan_path)
    pinfo = plan.info()
    assert pinfo["n"] == g.n and pinfo["m"] == g.m
    log(f"rank {rank}: plan ready in {time.time() - t0:.1f}s (hierarchy build "
        f"{pinfo['ch_seconds']:.1f}s, {pinfo['ch_up_arcs'] + pinfo['ch_dn_arcs']} arcs, levels "
        f"{pinfo['levels_up']}+{pinfo['levels_dn']})")

    dev = cpd.Graph(plan, device=gpu, batch=args.batch)
    # every rank builds the same number of rows per step (weak scaling): the
    # smallest batch any rank's free HBM allows
    (bmin,) = comm.reduce([float(dev.batch)], "MIN")
    if int(bmin) != dev.batch:
        dev.set_batch(int(bmin))
    B = dev.batch
    owned = shard_targets(g.n, world, args.partmethod, args.partkey, rank)
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
        rows = dev.build_rows(batch_of(owned, B, args.warmup + i), reuse=rows)
    comm.barrier()
    elapsed = time.perf_counter() - t0
    (elapsed_max,) = comm.reduce([elapsed], "MAX")
    kt = dev.timing_get()
    dev.timing(False)
    nrows, nruns = rows.count()
    last_targets = batch_of(owned, B, args.warmup + args.steps - 1)

    # ---- table-search on the last batch's rows ------------------------------
    ix = cpd.Index(dev, rows=rows)
    rng = np.random.default_rng(100 + rank)
    nq = args.queries
    qs = rng.integers(0, g.n, nq).astype(np.uint32)
    qt = last_targets[rng.integers(0, len(last_targets), nq)]
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

    q_rle, q_rle_ms = time_queries("rle")
    q_totals, q_ms_max = time_queries("auto")
    index_mode = ix.mode
    # congested leg (configs[2]): the .diff stand-in of SURVEY.md §8d — 10% of
    # edges x U[1, 3], rounded up — sent with the batch as fifo_auto does
    w_cong = cpd.synth_congestion(g.w, frac=0.1, lo=1.0, hi=3.0, seed=3)
    ix.set_weights(w_cong)
    q_cong, q_cong_ms = time_queries("auto")
    ix.set_weights(None)

    # ---- CPU baseline + full-size parity sample (rank 0, N = 1) -------------
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        sample = batch_of(owned, B, 0)[: threads * args.cpu_rows_per_thread]
        order = plan.order()
        tc = time.perf_counter()
        ref_off, ref_runs = oracle.build_rows(g.row_ptr, g.dst, g.w, order, sample, threads=threads)
        cpu_s = time.perf_counter() - tc
        grows = dev.build_rows(sample)
        goff, gruns = grows.export()
        parity = bool(np.array_equal(goff, ref_off) and np.array_equal(gruns, ref_runs))
        cq = 20000
        cs = rng.integers(0, g.n, cq).astype(np.uint32)
        ct = sample[rng.integers(0, len(sample), cq)]
        tq = time.perf_counter()
        rc, rh, rf = oracle.table_search(g.row_ptr, g.dst, g.w, order, sample, ref_off, ref_runs,
                                         cs, ct, threads=threads)
        cpu_q_s = time.perf_counter() - tq
        gix = cpd.Index(dev, rows=grows)
        gc, gh, gf, _ = gix.query(cs, ct)
        parity = parity and bool(np.array_equal(gc, rc) and np.array_equal(gh, rh))
        rcc, rch, _ = oracle.table_search(g.row_ptr, g.dst, w_cong, order, sample, ref_off,
                                          ref_runs, cs, ct, threads=threads)
        gix.set_weights(w_cong)
        gcc, gch, _, _ = gix.query(cs, ct)
        parity = parity and bool(np.array_equal(gcc, rcc) and np.array_equal(gch, rch))
        cpu = {"value": round(len(sample) / cpu_s, 3), "unit": "sources/s", "cores": threads,
               "kind": "port",
               "sample": f"{len(sample)} CPD rows of the same graph and partition (reverse Dijkstra "
                         f"+ first moves + RLE, C oracle, OpenMP {threads} threads, {cpu_s:.1f}s); "
                         f"table-search {cq} queries in {cpu_q_s:.2f}s",
               "queries_per_s": round(cq / cpu_q_s, 1)}

    if rank == 0:
        out = assemble(args, world, (g.n, g.m), B, elapsed_max, q_totals, q_ms_max, nrows, nruns,
                       kt, cpu, parity, pinfo, traffic)
        out["query_index"] = index_mode
        out["queries_per_s_rle"] = round(q_rle[0] / (q_rle_ms / 1e3), 1) if q_rle_ms else 0.0
        out["queries_per_s_congested"] = (round(q_cong[0] / (q_cong_ms / 1e3), 1)
                                          if q_cong_ms else 0.0)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
