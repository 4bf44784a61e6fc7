#!/usr/bin/env python3
"""Per-(kernel, grid) duration statistics from a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats groups dispatches by kernel name only; the averaging kernel runs at several
sizes under one name (grid = spans of 64 lanes), so this splits them by grid size and names the
element count each grid covers (fp32: 4 per lane, bf16: 8 per lane).

  python tools/trace_stats.py gpurun_out/cold_prof/cold_kernel_trace.csv [--match k_lerp] > profiles/x.csv
  python tools/trace_stats.py trace.csv --runs --pair-with k_stream_mix   # bench.py's interleaved cold launches
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
    ap.add_argument("--pair-with", default=None,
                    help="with --runs: a dispatch immediately followed by one of this kernel (same grid) belongs to "
                         "the group 'interleaved' (bench.py's cold launches, each followed by its access mix alone), "
                         "and those mix dispatches form their own group")
    args = ap.parse_args()
    groups = {}
    with open(args.trace) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    run_id, last_key = 0, None
    paired = set()
    if args.runs and args.pair_with:
        for i, row in enumerate(rows[:-1]):
            nxt = rows[i + 1]
            if args.pair_with in nxt["Kernel_Name"] and nxt["Grid_Size_X"] == row["Grid_Size_X"]:
                paired.add(i)
                paired.add(i + 1)
    for i, row in enumerate(rows):
        name = row["Kernel_Name"]
        key = (name, int(row["Grid_Size_X"]), int(row["Workgroup_Size_X"]))
        if i in paired:     # one group per kernel: the interleaved cold launches
            if args.match not in name and args.pair_with not in name:
                continue
            groups.setdefault(key + ("interleaved",), []).append(
                int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
            last_key = None
            continue
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
                "MaxNs", "StdDev", "Run"])
    for key, d in sorted(groups.items(), key=lambda kv: (kv[0][0], kv[0][1]) + tuple(str(x) for x in kv[0][3:])):
        name, grid, wg = key[:3]
        d = d[args.skip_first:] or d
        per_lane = 8 if "BF16" in name else 4
        w.writerow([name, grid, wg, grid * per_lane, len(d), round(sum(d) / len(d), 1), statistics.median(d), min(d),
                    max(d), round(statistics.pstdev(d), 1), key[3] if len(key) > 3 else ""])


if __name__ == "__main__":
    main()
