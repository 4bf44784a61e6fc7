#!/usr/bin/env python3
"""Whole gossip rounds of G co-resident resident learners on one GPU (tooling, not part of the
product): G = 2, 3, 4 and 8 learners of 11.17M fp32, fetch_probability 1, constant 0.5, their
averages batched (update_wait_average_many), timed like bench.py's round_sweep.  Every learner picks
another learner of the same process, so each round's dispatch is a closed group (k_lerp_pair /
k_lerp_group); DPWA_PAIR_FUSED=0 runs the same rounds on the XCD-grouped batch for an A/B.
Prints the averaged GB/s (3*N*s per averaging, bench.py's unit) and the round time per G."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dpwa_amd import DpwaConnection  # noqa: E402
from dpwa_amd.group import LocalGroup  # noqa: E402

N = bench.RESNET18_NUMEL
DEV = torch.device("cuda", 0)


def run(G, seconds=0.4):
    tmp = tempfile.mkdtemp()
    names = ["w%d" % (g + 1) for g in range(G)]
    cfg = os.path.join(tmp, "group.yaml")
    bench.write_config(cfg, names, "constant", 1.0, 0.0)
    group = LocalGroup()
    conns = [DpwaConnection(nm, cfg, seed=1000 + g, group=group) for g, nm in enumerate(names)]
    for g, c in enumerate(conns):
        t = torch.empty(N, device=DEV)
        t.normal_(generator=torch.Generator(device=DEV).manual_seed(g))
        c.make_resident(t)
    flats = [c.parameters for c in conns]
    losses = [1.0] * G

    def step():
        for c, f in zip(conns, flats):
            c.update_send(f, 1.0, reuse_snapshot=True)
        res = DpwaConnection.update_wait_average_many(conns, flats, losses)
        flats[:] = [c.parameters for c in conns]
        return sum(p is not None for p, _ in res)

    for _ in range(50):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    k = int(max(20, seconds / max(time.perf_counter() - t0, 1e-6)))
    t0 = time.perf_counter()
    averaged = sum(step() for _ in range(k))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for c in conns:
        c.close()
    torch.cuda.empty_cache()
    return averaged * 3 * N * 4 / el / 1e9, 1e6 * el / k, averaged / k


def main():
    for G in (2, 3, 4, 8):
        gbs, us, avg = run(G)
        print("G %d: %.1f GB/s averaged, %.2f us per round, %.2f averages per round" % (G, gbs, us, avg), flush=True)


if __name__ == "__main__":
    main()
