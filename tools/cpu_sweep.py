#!/usr/bin/env python3
"""CPU baselines of the averaging arithmetic at every north_star size (CPU
baseline (2)), on the host cores of the machine it runs on (the GPU box: same host as the
bench).  Per size, a bounded number of rounds of:
  * c_oracle  -- oracle/dpwa_oracle.c's fp32 (bf16) lerp, one thread (the restated
                 reference arithmetic, separate roundings), up to --c-oracle-max-numel;
  * torch_cpu -- the reference's statement itself (dpwa/adapters/pytorch.py:68,
                 factor*t + (1-factor)*p as torch eager ops) on every thread torch uses;
                 bf16 for the bf16 configs (torch-eager rounding, the bf16 extension).
Reported like bench.py's value: 3*N*s averaged bytes per round / time.  One JSON line per
measurement.  Usage: python tools/cpu_sweep.py [--max-seconds S] > out.jsonl
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = [(11_173_962, "f32"), (100_000_000, "f32"), (1_000_000_000, "bf16"), (7_000_000_000, "bf16")]


def timed(fn, max_seconds, min_rounds=1):
    rounds, t0 = 0, time.perf_counter()
    while True:
        fn()
        rounds += 1
        el = time.perf_counter() - t0
        if el >= max_seconds and rounds >= min_rounds:
            return rounds, el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-seconds", type=float, default=4.0)
    ap.add_argument("--c-oracle-max-numel", type=int, default=1_000_000_000)
    ap.add_argument("--max-numel", type=int, default=7_000_000_000)
    args = ap.parse_args()
    from oracle import lerp as olerp
    lib = olerp.clib()
    threads = torch.get_num_threads()
    for numel, dt in SIZES:
        if numel > args.max_numel:
            continue
        esize = 4 if dt == "f32" else 2
        g = torch.Generator().manual_seed(0)
        tdtype = torch.float32 if dt == "f32" else torch.bfloat16
        p = torch.empty(numel, dtype=tdtype).uniform_(-1.0, 1.0, generator=g)
        q = torch.empty(numel, dtype=tdtype).uniform_(-1.0, 1.0, generator=g)
        box = [p]

        def torch_round():
            box[0] = 0.5 * q + (1.0 - 0.5) * box[0]

        rounds, el = timed(torch_round, args.max_seconds)
        print(json.dumps({"numel": numel, "dtype": dt, "kind": "torch_cpu", "cores": threads, "rounds": rounds,
                          "seconds": round(el, 3), "ms_per_round": round(1e3 * el / rounds, 3),
                          "gbs": round(rounds * 3 * numel * esize / el / 1e9, 3)}), flush=True)
        box[0] = None
        if numel <= args.c_oracle_max_numel:
            fn = lib.dpwa_oracle_lerp_f32 if dt == "f32" else lib.dpwa_oracle_lerp_bf16
            pa, qa = p.data_ptr(), q.data_ptr()

            def c_round():
                fn(pa, qa, numel, 0.5)

            rounds, el = timed(c_round, args.max_seconds)
            print(json.dumps({"numel": numel, "dtype": dt, "kind": "c_oracle", "cores": 1, "rounds": rounds,
                              "seconds": round(el, 3), "ms_per_round": round(1e3 * el / rounds, 3),
                              "gbs": round(rounds * 3 * numel * esize / el / 1e9, 3)}), flush=True)
        del p, q, box


if __name__ == "__main__":
    main()
