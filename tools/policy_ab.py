#!/usr/bin/env python3
"""Interleaved A/B of the averaging kernel's cache policy (DPWA_LERP_POLICY, kernels.hip
LerpPolicy) on bench.py's N=1 line: each pass runs every policy once as its own process; prints one
JSON line per run (value, in-loop and cold kernel time, frac) and a summary of medians.

  python tools/policy_ab.py --policies 8,0,16 --passes 2 -- --steps 2000 --warmup 20
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = ["--no-cpu-baseline", "--no-sweep", "--compute-us", "0", "--no-secondary", "--no-parity"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--policies", default="8,0")
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--env", default="DPWA_LERP_POLICY")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    extra = [a for a in args.rest if a != "--"]
    res = {}
    for p in range(args.passes):
        for pol in args.policies.split(","):
            env = dict(os.environ, **{args.env: pol})
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + BASE + extra, env=env, cwd=ROOT,
                                 stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
            if out.returncode != 0:
                print(json.dumps({"policy": pol, "error": out.stderr[-500:]}), flush=True)
                continue
            d = json.loads(out.stdout.strip().splitlines()[-1])
            r = d["roofline"]
            row = {"pass": p, "policy": pol, "value": d["value"], "ms_per_step": d["ms_per_step"],
                   "in_loop_us": r["in_loop_avg_launch_us"], "cold_us": r["avg_launch_us"], "frac": r["frac"],
                   "value_cold": (d.get("value_cold") or {}).get("value")}
            res.setdefault(pol, []).append(row)
            print(json.dumps(row), flush=True)
    summary = {pol: {k: statistics.median([x[k] for x in rows if x[k] is not None] or [0])
                     for k in ("value", "ms_per_step", "in_loop_us", "cold_us", "frac", "value_cold")}
               for pol, rows in res.items()}
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    main()
