#!/usr/bin/env python3
"""Counters of the CPD-heuristic search kernels: runs
tools_scripts/search_ab.py (fscale 0 by default, a smaller query count)
under rocprofv3, one pass per counter group (at most 8 SQ / 4 TCC counters a
pass, MI355X_MICROARCH.md), and prints the sums over every cpd_search
dispatch plus the derived figures:

  vmem_rd_per_wave_cycle  SQ_INSTS_VMEM_RD / SQ_WAVE_CYCLES (quad-cycles)
  wait_frac               SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on memory)
  l2_hit_rate             TCC_HIT / (TCC_HIT + TCC_MISS)
  l2_latency              TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ (cycles)

  python tools_scripts/search_pmc.py OUT.json [search_ab args...]
"""
import csv
import glob
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
     "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VALU"],
    ["SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU",
     "SQ_ACTIVE_INST_VMEM", "SQ_INST_CYCLES_VMEM_RD", "SQ_INSTS_BRANCH"],
    ["TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum"],
    ["TCP_TCC_READ_REQ_sum", "TCP_TCC_READ_REQ_LATENCY_sum", "TCC_EA0_WRREQ_sum",
     "TCC_ATOMIC_sum"],
]


def main():
    out_path = sys.argv[1]
    extra = sys.argv[2:] or ["--fscale", "0", "--queries", "16384"]
    base = tempfile.mkdtemp(prefix="searchpmc-")
    res = {}
    for i, counters in enumerate(PASSES):
        d = os.path.join(base, f"p{i}")
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", *counters, "-d", d,
               "--output-format", "csv", "--", sys.executable,
               os.path.join(ROOT, "tools_scripts", "search_ab.py"), *extra]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           cwd=base)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if p.returncode or not files:
            print(f"pass {i} failed rc={p.returncode}: {p.stderr[-800:]}", file=sys.stderr)
            sys.exit(1)
        print(f"pass {i} done: {p.stdout.strip()[:200]}", flush=True)
        for row in csv.DictReader(open(files[0])):
            if "cpd_search" not in row["Kernel_Name"]:
                continue
            k = row["Counter_Name"]
            res[k] = res.get(k, 0.0) + float(row["Counter_Value"])
    g = lambda k: res.get(k, 0.0)
    der = {
        "vmem_rd_per_wave_cycle": g("SQ_INSTS_VMEM_RD") / max(1.0, g("SQ_WAVE_CYCLES")),
        "wait_frac": g("SQ_WAIT_ANY") / max(1.0, g("SQ_WAVE_CYCLES")),
        "active_frac": g("SQ_ACTIVE_INST_ANY") / max(1.0, g("SQ_WAVE_CYCLES")),
        "l2_hit_rate": g("TCC_HIT_sum") / max(1.0, g("TCC_HIT_sum") + g("TCC_MISS_sum")),
        "l2_latency": g("TCP_TCC_READ_REQ_LATENCY_sum") / max(1.0, g("TCP_TCC_READ_REQ_sum")),
        "dram_frac": g("TCC_EA0_RDREQ_DRAM_sum") / max(1.0, g("TCC_EA0_RDREQ_sum")),
    }
    out = {"args": extra, "counters": res, "derived": der}
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(der))


if __name__ == "__main__":
    main()
