#!/usr/bin/env python3
"""Overlap of the early up-sweep with first moves, from a rocprofv3
kernel-trace CSV: for each first_moves launch, the share of its interval
during which some sweep_up kernel ran; and the step timeline.

  python tools_scripts/overlap_trace.py gpurun_out/trace_TAG/**/kernel_trace.csv
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = []
    for r in rows:
        n = r["Kernel_Name"]
        tag = ("up" if "sweep_up" in n else "down" if "sweep_down8" in n else
               "fm" if "first_moves" in n else "emit" if "rle_scan<true" in n else
               "count" if "rle_count_ch" in n else None)
        if tag:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), tag,
                       r.get("Queue_Id", r.get("Stream_Id", ""))))
    ks.sort()
    fms = [k for k in ks if k[2] == "fm"]
    ups = [k for k in ks if k[2] == "up"]
    for a, b, _, q in fms:
        cov = 0
        for c, d, _, _ in ups:
            lo, hi = max(a, c), min(b, d)
            if hi > lo:
                cov += hi - lo
        up_in = [u for u in ups if u[0] < b and u[1] > a]
        print(f"fm {(b - a) / 1e6:.2f} ms queue {q}: up kernels overlapping {len(up_in)}, "
              f"covered {cov / max(1, b - a):.2f}")
    print("queues:", sorted({(k[2], k[3]) for k in ks}))


if __name__ == "__main__":
    main()
