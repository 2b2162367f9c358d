"""Summarise a rocprofv3 --kernel-trace --stats run next to the bench line it
profiled: per kernel calls / total / average device time from rocprofv3, and
the bench's own HIP-event averages for the same kernels (they must agree)."""
import csv
import glob
import json
import sys

# most specific first: rocprof names carry template arguments
NAMES = [("DenseRows", "table_search_dense"), ("RleRows", "table_search"),
         ("validate_rows", "validate_rows"), ("sweep_down8", "sweep_down"), ("first_moves_n4", "first_moves"),
         ("count_wide_rows", "wide_rows_count"), ("target_mask", "target_mask"),
         ("sweep_up_sparse", "sweep_up"), ("sweep_up_chunks", "sweep_up"),
         ("sweep_up_init", "sweep_up_init"), ("sweep_level<true>", "sweep_up"),
         ("sweep_level<false>", "sweep_down"), ("first_moves", "first_moves"),
         ("rle_scan<false", "rle_count"), ("rle_scan<true", "rle_emit"),
         ("table_search_dense", "table_search_dense"), ("table_search", "table_search"),
         ("expand_rows", "expand_rows"), ("live_stats", "live_stats")]


def main(prof_dir, bench_json, out_md):
    stats = glob.glob(f"{prof_dir}/**/*kernel_stats.csv", recursive=True)[0]
    bench = json.load(open(bench_json))
    lines = ["| kernel | rocprof calls | rocprof avg µs | rocprof total ms | bench launches | bench avg µs |",
             "|---|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats)):
        short = next((v for k, v in NAMES if k in r["Name"]), r["Name"][:40])
        b = bench.get("kernels", {}).get(short)
        bavg = f"{b['ms'] * 1e3 / b['launches']:.1f}" if b else "-"
        bl = b["launches"] if b else "-"
        lines.append(f"| {short} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.2f} | {bl} | {bavg} |")
    open(out_md, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:4])
