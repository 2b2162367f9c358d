#!/usr/bin/env python3
"""L2 / fabric counters of the table-search walk.

Runs bench.py's PMC child (one build step + one 1M-query dense walk of the
synth1m workload; needs the bench's plan cache, so run after bench.py on the
same box) under rocprofv3, one pass per counter group (a TCC pass holds at
most 4 TCC counters, MI355X_MICROARCH.md), and prints per-kernel sums:

  l2_hit_rate   TCC_HIT / (TCC_HIT + TCC_MISS)
  ea_rdreq      L2 -> fabric read requests (Infinity Cache or HBM), by size
  dram_rdreq    of those, requests that went to DRAM
  l2_latency    TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ (cycles)

  python tools_scripts/walk_pmc.py OUT.json
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ["TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum"],
    ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_REQ_sum"],
    ["TCP_TCC_READ_REQ_sum", "TCP_TCC_READ_REQ_LATENCY_sum"],
]
KERNELS = {"DenseRows": "table_walk_dense", "first_moves_n4": "first_moves",
           "sweep_down8": "sweep_down", "rle_scan<true": "rle_emit", "expand_rows": "expand_rows"}


def main():
    out_path = sys.argv[1]
    base = tempfile.mkdtemp(prefix="walkpmc-")
    res = {}
    for i, counters in enumerate(PASSES):
        d = os.path.join(base, f"p{i}")
        cmd = ["timeout", "-s", "KILL", "180", "rocprofv3", "--pmc", *counters, "-d", d,
               "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "bench.py"),
               "--pmc-child", "--steps", "1", "--warmup", "0"]
        p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                           cwd=base)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if p.returncode or not files:
            print(f"pass {i} failed rc={p.returncode}: {p.stderr[-500:]}", file=sys.stderr)
            sys.exit(1)
        for row in csv.DictReader(open(files[0])):
            k = next((v for kk, v in KERNELS.items() if kk in row["Kernel_Name"]), None)
            if k is None:
                continue
            e = res.setdefault(k, {})
            e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    for k, e in res.items():
        h, m = e.get("TCC_HIT_sum", 0.0), e.get("TCC_MISS_sum", 0.0)
        e["l2_hit_rate"] = round(h / (h + m), 4) if h + m else None
        rq = e.get("TCP_TCC_READ_REQ_sum", 0.0)
        e["l2_latency_cycles"] = round(e.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / rq, 1) if rq else None
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res))
    shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
