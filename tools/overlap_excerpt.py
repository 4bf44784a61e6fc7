#!/usr/bin/env python3
"""Cuts a rocprofv3 kernel trace of tools/overlap_trace.py down to the kernels around a few
side-stream pulls (k_pull) -- enough to see each pull next to the training step's kernels --
so the evidence fits in profiles/.  Usage: overlap_excerpt.py <trace_dir> <out.csv> [pulls]"""
import csv
import glob
import os
import sys


def main():
    trace_dir, out = sys.argv[1], sys.argv[2]
    want = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    fn = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(fn)), key=lambda r: int(r["Start_Timestamp"]))
    pulls = [i for i, r in enumerate(rows) if "k_pull" in r["Kernel_Name"]]
    picks = pulls[len(pulls) // 2:len(pulls) // 2 + want]
    keep = sorted({j for i in picks for j in range(max(0, i - 8), min(len(rows), i + 12))})
    t0 = int(rows[keep[0]]["Start_Timestamp"])
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["start_us", "end_us", "queue", "kernel"])
        for j in keep:
            r = rows[j]
            w.writerow([round((int(r["Start_Timestamp"]) - t0) / 1e3, 3), round((int(r["End_Timestamp"]) - t0) / 1e3, 3),
                        r["Queue_Id"], r["Kernel_Name"][:90]])


if __name__ == "__main__":
    main()
