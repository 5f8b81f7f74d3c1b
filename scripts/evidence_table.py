#!/usr/bin/env python3
"""Markdown rows of DESIGN.md §6's measurement table from one round's evidence directory (scripts/gpu_r6_evidence.sh
output: <dir>/<query>/bench.json, pmc.json, prof/bench_kt/kt_kernel_stats.csv).

    python3 scripts/evidence_table.py gpurun_out/r6e c2 c2real ...
"""
import csv
import json
import os
import sys


def kernel_avg_ms(d):
    """rocprofv3 average duration of the scan kernels (scan_lean / scan_tiles instantiations, summed per query)."""
    p = os.path.join(d, "prof", "bench_kt", "kt_kernel_stats.csv")
    if not os.path.exists(p):
        return None
    tot = 0.0
    for row in csv.DictReader(open(p)):
        if "scan_lean" in row["Name"] or "scan_tiles" in row["Name"] or "ex_scan" in row["Name"]:
            tot += float(row["AverageNs"]) / 1e6
    return tot or None


def main(root, queries):
    for q in queries:
        d = os.path.join(root, q)
        b = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
        rf = b["roofline"]
        pmc = None
        if os.path.exists(os.path.join(d, "pmc.json")):
            pmc = json.load(open(os.path.join(d, "pmc.json")))
        kt = kernel_avg_ms(d)
        v = b.get("validated") or {}
        traffic = (f"{pmc['hbm_read_bytes_per_launch'] / 1e9:.2f} + {pmc['write_size_bytes_raw'] / 1e9:.3f}"
                   if pmc else "—")
        print(f"| {q} | {b['scan_kernel_ms']:.3f} ms" + (f" ({kt:.3f})" if kt else "") +
              f" | {b['eval_ms']:.3f} ms | {b['cold_eval_ms']:.2f} ms | {rf['plan_bytes_per_launch'] / 1e9:.2f} | "
              f"{rf['frac']:.3f} | {rf.get('frac_algorithmic', 0):.2f} | {traffic} | {b['output_rows']:,} | "
              f"{b['value']:.3g} | {'ok' if v.get('ok') else v} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
