#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 kernel-trace CSV: for one
steady-state step (first_moves start to the next first_moves start), each
kernel family's launches, busy time and span per queue, and the time the
GPU ran nothing.   python tools_scripts/step_timeline.py TRACE.csv [step]"""
import csv
import sys
from collections import defaultdict

FAMILIES = [("sweep_up_sparse", "up_sparse"), ("sweep_up_chunks", "up_chunks"),
            ("sweep_up_init", "up_init"), ("sweep_down8", "down"), ("first_moves", "fm"),
            ("rle_moves", "moves"), ("rle_count", "count"), ("rle_fix", "fix"),
            ("rle_scan", "rle_scan"), ("live_stats", "live")]


def family(name):
    for key, tag in FAMILIES:
        if key in name:
            return tag
    return name.split("(")[0][-32:]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"]),
                 r["Queue_Id"]) for r in rows)
    fms = [k for k in ks if k[2] == "fm"]
    si = int(sys.argv[2]) if len(sys.argv) > 2 else len(fms) // 2
    a, b = fms[si][0], fms[si + 1][0]
    step = [k for k in ks if k[1] > a and k[0] < b]
    agg = defaultdict(lambda: [0, 0, 1e30, 0])
    for s, e, t, q in step:
        s2, e2 = max(s, a), min(e, b)
        g = agg[(t, q)]
        g[0] += 1
        g[1] += e2 - s2
        g[2] = min(g[2], s2)
        g[3] = max(g[3], e2)
    print(f"step {si}: {(b - a) / 1e6:.2f} ms")
    for (t, q), g in sorted(agg.items(), key=lambda x: x[1][2]):
        print(f"  {t:14s} q{q:>3} n={g[0]:4d} busy {g[1] / 1e6:7.2f} ms  {(g[2] - a) / 1e6:7.2f} -> {(g[3] - a) / 1e6:7.2f}")
    iv = sorted((max(s, a), min(e, b)) for s, e, _, _ in step)
    busy, cur = 0, None
    for s, e in iv:
        if cur is None or s > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        busy += cur[1] - cur[0]
    print(f"  idle {(b - a - busy) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
