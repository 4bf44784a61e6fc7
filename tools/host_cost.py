#!/usr/bin/env python3
"""Host cost of one N=1 resident gossip round, by part (tooling, not part of the product).

bench.py's timed window is 20 rounds after a synchronize: if a round's host enqueue is not well
under its ~27 us dispatch, the window runs host-bound.  Times, per round, update_send of both
learners, update_wait_average_many and the two `parameters` reads -- (a) with the GPU drained
before every round (no back-pressure: the host's own cost), (b) free-running (steady state), and
(c) the first 20 rounds after a synchronize, as bench.py's timed window runs them."""
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

N = int(os.environ.get("HOST_COST_NUMEL", bench.RESNET18_NUMEL))
DEV = torch.device("cuda", 0)


def main():
    tmp = tempfile.mkdtemp()
    cfg = os.path.join(tmp, "bench.yaml")
    bench.write_config(cfg, ["w1", "w2"], "constant", 1.0, 0.0)
    group = LocalGroup()
    conns = [DpwaConnection(nm, cfg, seed=1000 + g, group=group) for g, nm in enumerate(("w1", "w2"))]
    for g, c in enumerate(conns):
        t = torch.empty(N, device=DEV)
        t.normal_(generator=torch.Generator(device=DEV).manual_seed(g))
        c.make_resident(t)
    flats = [c.parameters for c in conns]
    pc = time.perf_counter

    def round_(parts):
        t0 = pc()
        for c, f in zip(conns, flats):
            c.update_send(f, 1.0, reuse_snapshot=True)
        t1 = pc()
        DpwaConnection.update_wait_average_many(conns, flats, [1.0, 1.0])
        t2 = pc()
        flats[:] = [c.parameters for c in conns]
        t3 = pc()
        parts.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))

    for _ in range(3000):
        round_([])
    torch.cuda.synchronize()
    # (a) drained before every round
    parts = []
    for _ in range(2000):
        torch.cuda.synchronize()
        round_(parts)
    a = np.array(parts) * 1e6
    print("drained   us: send %.2f  wait_many %.2f  params %.2f  round %.2f  (median; p90 round %.2f)"
          % tuple(list(np.median(a, axis=0)) + [np.percentile(a[:, 3], 90)]), flush=True)
    # (b) free-running
    parts = []
    torch.cuda.synchronize()
    t0 = pc()
    for _ in range(4000):
        round_(parts)
    host = pc() - t0
    torch.cuda.synchronize()
    tot = pc() - t0
    a = np.array(parts) * 1e6
    print("free      us: send %.2f  wait_many %.2f  params %.2f  round %.2f  (median)  host/round %.2f  "
          "total/round %.2f" % tuple(list(np.median(a, axis=0)) + [1e6 * host / 4000, 1e6 * tot / 4000]), flush=True)
    # (c) bench's window: 20 rounds after a synchronize (+ a 1 ms host pause, like a barrier)
    wins, per_round = [], []
    for _ in range(200):
        torch.cuda.synchronize()
        time.sleep(0.001)
        torch.cuda.synchronize()
        parts = []
        t0 = pc()
        for _ in range(20):
            round_(parts)
        torch.cuda.synchronize()
        wins.append((pc() - t0) / 20 * 1e6)
        per_round.append([p[3] * 1e6 for p in parts])
    pr = np.median(np.array(per_round), axis=0)
    print("window    us/round: median %.2f  p10 %.2f  p90 %.2f; host per round by position: %s"
          % (np.median(wins), np.percentile(wins, 10), np.percentile(wins, 90), " ".join("%.1f" % x for x in pr)),
          flush=True)
    for c in conns:
        c.close()


if __name__ == "__main__":
    main()
