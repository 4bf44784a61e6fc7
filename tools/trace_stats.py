#!/usr/bin/env python3
"""Per-(kernel, grid) duration statistics from a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats groups dispatches by kernel name only; the averaging kernel runs at several
sizes under one name (grid = spans of 64 lanes), so this splits them by grid size and names the
element count each grid covers (fp32: 4 per lane, bf16: 8 per lane).

  python tools/trace_stats.py gpurun_out/cold_prof/cold_kernel_trace.csv [--match k_lerp] > profiles/x.csv
"""
import argparse
import csv
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="k_lerp")
    ap.add_argument("--skip-first", type=int, default=0, help="drop the first k dispatches of each group (warmup)")
    ap.add_argument("--runs", action="store_true",
                    help="split each (kernel, grid) group into runs of consecutive dispatches (a dispatch of any "
                         "other kernel ends a run): e.g. bench.py's timed loop and its cold measurement")
    args = ap.parse_args()
    groups = {}
    with open(args.trace) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    run_id, last_key = 0, None
    for row in rows:
        name = row["Kernel_Name"]
        key = (name, int(row["Grid_Size_X"]), int(row["Workgroup_Size_X"]))
        if key != last_key:
            run_id += 1
            last_key = key
        if args.match not in name:
            continue
        if args.runs:
            key = key + (run_id,)
        groups.setdefault(key, []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "GridThreads", "WorkgroupSize", "ElementsCovered", "Calls", "AverageNs", "MedianNs", "MinNs",
                "MaxNs", "StdDev"])
    for key, d in sorted(groups.items(), key=lambda kv: (kv[0][0], kv[0][1]) + tuple(kv[0][3:])):
        name, grid, wg = key[:3]
        d = d[args.skip_first:] or d
        per_lane = 8 if "BF16" in name else 4
        w.writerow([name, grid, wg, grid * per_lane, len(d), round(sum(d) / len(d), 1), statistics.median(d), min(d),
                    max(d), round(statistics.pstdev(d), 1)])


if __name__ == "__main__":
    main()
