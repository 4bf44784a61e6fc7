#!/usr/bin/env python3
"""Why does bench.py's timed N=1 loop run the resident pair slower than its round sweep? (tooling,
not part of the product).  Times 2000 gossip rounds of two co-resident resident learners through
the connection API in variants that differ in one respect each from bench.py's main loop:
initial data (randn vs normal_), update_send's reuse flag, update_wait_average_many's write-through
flag, the interpolation config file, and fresh vs reused learners."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from dpwa_amd import DpwaConnection  # noqa: E402
from dpwa_amd.group import LocalGroup  # noqa: E402

N = bench.RESNET18_NUMEL
K = int(os.environ.get("PAIR_DIAG_ROUNDS", "2000"))
DEV = torch.device("cuda", 0)


def make(cfg, data):
    group = LocalGroup()
    conns = [DpwaConnection(nm, cfg, seed=1000 + g, group=group) for g, nm in enumerate(("w1", "w2"))]
    for g, c in enumerate(conns):
        if data == "randn":
            t = torch.randn(N, device=DEV, generator=torch.Generator(device=DEV).manual_seed(g), dtype=torch.float32)
        else:
            t = torch.empty(N, device=DEV)
            t.normal_(generator=torch.Generator(device=DEV).manual_seed(g))
        c.make_resident(t)
    return conns


HOST = []


def rounds(conns, k, reuse, wt):
    flats = [c.parameters for c in conns]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        for c, f in zip(conns, flats):
            c.update_send(f, 1.0, reuse_snapshot=reuse)
        DpwaConnection.update_wait_average_many(conns, flats, [1.0, 1.0], write_through=wt)
        flats[:] = [c.parameters for c in conns]
    HOST.append(1e6 * (time.perf_counter() - t0) / k)      # host time per round (enqueue only)
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / k


def addrs(conns):
    import ctypes
    from dpwa_amd import _lib
    out = []
    for c in conns:
        for k in (0, 1):
            c.parameters      # (resident pointer)
        p = ctypes.c_void_p()
        _lib.call("dpwa_learner_resident_params", c._learner.handle, ctypes.byref(p), None)
        out.append(p.value)
    return out


def main():
    tmp = tempfile.mkdtemp()
    cfg = os.path.join(tmp, "bench.yaml")
    bench.write_config(cfg, ["w1", "w2"], "constant", 1.0, 0.0)
    keep = []
    for it in range(8):       # fresh pairs, the old ones kept alive (even it) or closed (odd it)
        conns = make(cfg, "normal")
        rounds(conns, 200, True, True)
        us = [rounds(conns, K, True, True) for _ in range(2)]
        a = addrs(conns)
        print("pair %d keep=%d us/round %s (host %.2f)  A %#x B %#x  B-A %+.1f MiB"
              % (it, it % 2 == 0, " ".join("%.2f" % u for u in us), HOST[-1], a[0], a[1], (a[1] - a[0]) / 2 ** 20),
              flush=True)
        if it % 2 == 0:
            keep.append(conns)
        else:
            for c in conns:
                c.close()
            torch.cuda.synchronize()
    for conns in keep:
        for c in conns:
            c.close()
    torch.cuda.synchronize()
    for variant in ("sweep-like", "randn", "reuse=False", "wt=False", "main-like", "sweep-like"):
        data = "randn" if variant in ("randn", "main-like") else "normal"
        reuse = variant not in ("reuse=False", "main-like")
        wt = variant not in ("wt=False", "main-like")
        conns = make(cfg, data)
        rounds(conns, 200, reuse, wt)
        us = [rounds(conns, K, reuse, wt) for _ in range(3)]
        print("%-12s us/round %s (host %.2f)" % (variant, " ".join("%.2f" % u for u in us), HOST[-1]), flush=True)
        for c in conns:
            c.close()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
