#!/usr/bin/env python3
"""A/B of the slot allocation behind the N=1 resident pair loop (tooling, not part of the
product): pairs of resident learners created alternately with hipMalloc, physically contiguous
slots (DPWA_CONTIG=1: hipExtMallocWithFlags(hipDeviceMallocContiguous)) and hipMemCreate chunks
(DPWA_VMM=1), each timed over 4000 free-running rounds (GPU-bound), in one process.
DPWA_CONTIG was a temporary knob in learner.cpp devmem_alloc for this A/B (removed: the spread it
showed follows the chip's state over time, profiles/r04_pair_state.md); without it that mode is
plain hipMalloc."""
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
MODES = {"hipMalloc": {}, "contiguous": {"DPWA_CONTIG": "1"}, "vmm": {"DPWA_VMM": "1"}}


def pair(cfg, env):
    for k in ("DPWA_CONTIG", "DPWA_VMM"):
        os.environ.pop(k, None)
    os.environ.update(env)
    group = LocalGroup()
    conns = [DpwaConnection(nm, cfg, seed=1000 + g, group=group) for g, nm in enumerate(("w1", "w2"))]
    for g, c in enumerate(conns):
        t = torch.empty(N, device=DEV)
        t.normal_(generator=torch.Generator(device=DEV).manual_seed(g))
        c.make_resident(t)
    for k in ("DPWA_CONTIG", "DPWA_VMM"):
        os.environ.pop(k, None)
    return conns


def rounds(conns, k):
    flats = [c.parameters for c in conns]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        for c, f in zip(conns, flats):
            c.update_send(f, 1.0, reuse_snapshot=True)
        DpwaConnection.update_wait_average_many(conns, flats, [1.0, 1.0])
        flats[:] = [c.parameters for c in conns]
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / k


def main():
    tmp = tempfile.mkdtemp()
    cfg = os.path.join(tmp, "bench.yaml")
    bench.write_config(cfg, ["w1", "w2"], "constant", 1.0, 0.0)
    res = {m: [] for m in MODES}
    passes = int(os.environ.get("ALLOC_AB_PASSES", "4"))
    for p in range(passes):
        for m, env in MODES.items():
            conns = pair(cfg, env)
            rounds(conns, 1000)
            us = rounds(conns, 4000)
            res[m].append(us)
            print("pass %d %-10s %.2f us/round" % (p, m, us), flush=True)
            for c in conns:
                c.close()
            torch.cuda.synchronize()
    for m, v in res.items():
        print("%-10s median %.2f  min %.2f  max %.2f us/round" % (m, np.median(v), min(v), max(v)), flush=True)


if __name__ == "__main__":
    main()
