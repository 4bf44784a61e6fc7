#!/usr/bin/env python3
"""Checks a bench.py stdout capture the way the driver reads it: exactly one non-empty line, at
most bench.LINE_MAX bytes, json.loads succeeds, the contract keys present, scalar blocks only,
and a completed run (no `error`, not the provisional N>1 line).
Prints a one-line summary.  Usage: tools/check_line.py <stdout file>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "config", "roofline", "scaling_basis")


def main(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.strip()]
    assert len(lines) == 1, "%d lines" % len(lines)
    n = len(lines[0].encode())
    assert n <= bench.LINE_MAX, "line is %d bytes" % n
    d = json.loads(lines[0])
    missing = [k for k in KEYS if k not in d]
    assert not missing, "missing %s" % missing
    for block in ("roofline", "config", "cpu_baseline", "parity", "xgmi"):
        if isinstance(d.get(block), dict):
            assert not any(isinstance(v, (dict, list)) for v in d[block].values()), block
    # a held line printed after a failure (watchdog, exception, signal) or the provisional one is
    # still a parseable line, but not a completed run
    assert "error" not in d and not d.get("provisional"), "not a completed run: %s" % d.get("error", "provisional")
    print("%s: %d bytes, n_gpus %s, value %s, ms_per_step %s, frac %s, pull %s, parity %s, weak %s" % (
        path, n, d["n_gpus"], d["value"], d["ms_per_step"], d["roofline"].get("frac"), d.get("pull"),
        "all true" if all((d.get("parity") or {"-": False}).values()) else d.get("parity"),
        d["scaling_basis"].get("weak", {}).get("gossip_rounds_per_s")))


if __name__ == "__main__":
    main(sys.argv[1])
