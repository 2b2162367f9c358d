#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per kernel name, and per sweep
dispatch index within a batch (= level order), the mean duration and grid."""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    # the bench process's trace (a plan-building child writes its own)
    f = max(files, key=lambda x: open(x).read().count("first_moves"))
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tot = defaultdict(lambda: [0, 0.0])
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        r["_n"] = name
        r["_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[name][0] += 1
        tot[name][1] += r["_us"]
    print("kernel                                   calls   total_ms   avg_us")
    for k, (c, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:40]:40s} {c:6d} {us / 1e3:10.2f} {us / c:8.1f}")
    # per level: sweeps between two first_moves launches form one batch
    for kind in ("sweep_up_sparse", "sweep_up_chunks", "sweep_down8", "sweep_level<false>", "sweep_level<true>"):
        per = defaultdict(list)
        idx = 0
        for r in rows:
            if "first_moves" in r["_n"]:
                idx = 0
            elif kind in r["_n"]:
                per[idx].append((r["_us"], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)))
                idx += 1
        if not per:
            continue
        print(f"\n{kind}: level-index  mean_us  grid  (cumulative ms per batch)")
        cum = 0.0
        nb = max(len(v) for v in per.values())
        for i in sorted(per):
            us = sum(x[0] for x in per[i]) / len(per[i])
            cum += us / 1e3
            if i < 25 or i % 10 == 0 or i == len(per) - 1 or us > 300:
                print(f"  {i:4d} {us:9.1f} {per[i][0][1]:10d}  {cum:8.2f}")
        print(f"  batches seen: {nb}")
    # the main stream between the down-sweep's levels: gaps from one level's
    # end to the next one's start, per batch (launch latency + tail drain)
    gaps, busy, prev = defaultdict(float), defaultdict(float), None
    b = 0
    for r in rows:
        if "first_moves" in r["_n"]:
            b += 1
            prev = None
        elif "sweep_down8" in r["_n"]:
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if prev is not None:
                gaps[b] += max(0, s0 - prev) / 1e6
            busy[b] += (e0 - s0) / 1e6
            prev = e0
    for k in sorted(gaps):
        print(f"batch {k}: down-sweep busy {busy[k]:.2f} ms, gaps between its levels {gaps[k]:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
