#!/usr/bin/env python3
"""Attributes the GPU's idle time between a run's averaging kernels to the host ranges that
were open meanwhile (SURVEY §5 tracing).  Input: a rocprofv3 `--marker-trace --kernel-trace`
directory of a run with DPWA_ROCTX=1 (dpwa_amd/csrc/trace.cpp ranges).

For each pair of consecutive launches of the dominant kernel (by count; or --kernel SUBSTR), the
gap [end_i, start_i+1] is split at every range boundary and each piece is charged to the
innermost dpwa range open at that time (the shortest one covering it), or to "(no dpwa range)"
-- host code above the library (Python, the bench loop).  Prints a JSON summary: per round, the
kernel time, the gap, and the gap by range; plus each range's mean host duration.
Usage: tools/marker_gaps.py <rocprofv3 output dir> [--kernel SUBSTR] [--skip N]"""
import argparse
import bisect
import csv
import glob
import json
import os
from collections import Counter, defaultdict


def _rows(d, suffix):
    paths = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    if not paths:
        raise SystemExit("no *%s under %s" % (suffix, d))
    out = []
    for p in paths:
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def analyse(d, kernel=None, skip=20):
    kt = _rows(d, "kernel_trace.csv")
    names = Counter(r["Kernel_Name"] for r in kt)
    if kernel:
        pick = [n for n in names if kernel in n]
        if not pick:
            raise SystemExit("no kernel matching %r" % kernel)
        kname = max(pick, key=names.get)
    else:
        kname = names.most_common(1)[0][0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt if r["Kernel_Name"] == kname)
    ks = ks[skip:]                        # the warmup rounds
    mk = _rows(d, "marker_api_trace.csv")
    ranges = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in mk)
    starts = [r[0] for r in ranges]
    by_range = defaultdict(float)
    gaps, kern = [], []
    for (s0, e0), (s1, _e1) in zip(ks, ks[1:]):
        kern.append(e0 - s0)
        if s1 <= e0:
            gaps.append(0)
            continue
        gaps.append(s1 - e0)
        # ranges that can overlap [e0, s1): started before s1 (ranges are short: look back a bit)
        hi = bisect.bisect_left(starts, s1)
        lo = bisect.bisect_left(starts, e0 - 50_000_000)
        cand = [r for r in ranges[lo:hi] if r[1] > e0]
        cuts = sorted({e0, s1} | {t for r in cand for t in (r[0], r[1]) if e0 < t < s1})
        for a, b in zip(cuts, cuts[1:]):
            mid = (a + b) / 2
            cover = [r for r in cand if r[0] <= mid < r[1]]
            name = min(cover, key=lambda r: r[1] - r[0])[2] if cover else "(no dpwa range)"
            by_range[name] += b - a
    n = max(1, len(gaps))
    dur = defaultdict(list)
    for s, e, name in ranges:
        dur[name].append(e - s)
    total_gap = sum(gaps)
    return {
        "kernel": kname[:160],
        "rounds": len(gaps),
        "kernel_us_mean": round(sum(kern) / max(1, len(kern)) / 1e3, 3),
        "gap_us_mean": round(total_gap / n / 1e3, 3),
        "gap_us_median": round(sorted(gaps)[len(gaps) // 2] / 1e3, 3) if gaps else None,
        "gap_by_range_us_per_round": {k: round(v / n / 1e3, 3)
                                      for k, v in sorted(by_range.items(), key=lambda kv: -kv[1])},
        "gap_share_by_range": {k: round(v / total_gap, 4) for k, v in sorted(by_range.items(), key=lambda kv: -kv[1])}
        if total_gap else {},
        "range_host_us_mean": {k: round(sum(v) / len(v) / 1e3, 3) for k, v in sorted(dur.items())},
        "range_calls": {k: len(v) for k, v in sorted(dur.items())},
        "note": "gap = GPU idle between consecutive launches of the kernel (rocprofv3 timestamps); each piece of it "
                "is charged to the innermost dpwa roctx range open on the host then; ranges and kernel times are "
                "under the profiler (its hooks slow the host)",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--skip", type=int, default=20)
    a = ap.parse_args()
    print(json.dumps(analyse(a.dir, a.kernel, a.skip), indent=1))


if __name__ == "__main__":
    main()
