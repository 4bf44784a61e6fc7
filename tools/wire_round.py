#!/usr/bin/env python3
"""f3 measurement: gossip rounds of GPU learners that speak the reference's TCP protocol
(dpwa_amd/bridge.py WireConnection: `<HLL` framing + pickle, conn.py:98-110 / messaging.py),
two learners in one process on one GPU over localhost, at BASELINE configs[1]'s size.

Each round: both update_send (publish into HBM; with eager=True the fetch starts on a
background thread, TxThread-style), then both update_wait_average (the fetched blob is staged
into HBM and averaged by the fused kernel).  Reports ms per round, averaged GB/s (3*N*s per
averaging) and the phases of one learner's fetch.  The reference's own CPU round over the same
protocol is bench.py's cpu_baseline (~100-120 ms at this size on the GPU box's host).

  python tools/wire_round.py [--numel 11173962] [--rounds 10] [--eager 1] > out.json
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dpwa_amd.bridge import SnapshotCodec, WireConnection   # noqa: E402


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


NAMES = ["wa", "wb"]


def _proc(g, cfg, args, barrier, results):
    """--procs 2: learner g in its own process (the reference runs one learner per process)."""
    dev = torch.device("cuda", 0)
    conn = WireConnection(NAMES[g], cfg, codec=SnapshotCodec.single("w", args.numel), seed=10 + g,
                          eager=bool(args.eager))
    flat = torch.randn(args.numel, device=dev, generator=torch.Generator(device=dev).manual_seed(g))

    def round_():
        conn.update_send(flat, 1.0)
        return conn.update_wait_average(flat, 1.0)[0] is not None

    conn.update_send(flat, 1.0)      # both learners have published before anyone fetches
    barrier.wait()
    conn.update_wait_average(flat, 1.0)
    for _ in range(args.warmup):
        round_()
    torch.cuda.synchronize()
    barrier.wait()
    times, averaged = [], 0
    for _ in range(args.rounds):
        t0 = time.perf_counter()
        averaged += round_()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    barrier.wait()                   # neither closes while the other may still fetch
    results.put((g, times, averaged))
    barrier.wait()
    conn.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=int, default=11_173_962)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--eager", type=int, default=1)
    ap.add_argument("--procs", type=int, default=1, choices=(1, 2), help="learners in one process or one each")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    names = NAMES
    ports = [free_port(), free_port()]
    tmp = tempfile.mkdtemp(prefix="dpwa_wire_")
    cfg = os.path.join(tmp, "wire.yaml")
    lines = ["- nodes:"] + ["  - {name: %s, host: 127.0.0.1, port: %d}" % (n, p) for n, p in zip(names, ports)]
    lines += ["- fetch_probability: 1.0", "- timeout_ms: 30000", "- interpolation: constant",
              "- divergence_threshold: 0", "- constant: { value: 0.5 }", "- clock: 0", "- loss: 0"]
    with open(cfg, "w") as f:
        f.write("\n".join(lines) + "\n")
    if args.procs == 2:
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        barrier, results = ctx.Barrier(2), ctx.Queue()
        ps = [ctx.Process(target=_proc, args=(g, cfg, args, barrier, results)) for g in range(2)]
        for p in ps:
            p.start()
        got = [results.get(timeout=600) for _ in ps]
        for p in ps:
            p.join(120)
        per = [t for _, t, _ in got]
        el = max(float(np.sum(t)) for t in per)
        averaged = sum(a for _, _, a in got)
        rounds = [float(np.median(t)) for t in per]
        print(json.dumps({
            "what": "two GPU learners, one process each, gossiping over the reference's TCP protocol "
                    "(WireConnection), one MI355X, localhost; fp32, constant 0.5, fetch_probability 1",
            "numel": args.numel, "eager_fetch": bool(args.eager), "procs": 2, "rounds": args.rounds,
            "averagings": averaged, "ms_per_round_median": round(1e3 * max(rounds), 2),
            "averaged_gbs": round(averaged * 3 * args.numel * 4 / el / 1e9, 3), "blob_bytes": args.numel * 4,
            "cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}))
        return
    conns = [WireConnection(names[g], cfg, codec=SnapshotCodec.single("w", args.numel), seed=10 + g,
                            eager=bool(args.eager)) for g in range(2)]
    flats = [torch.randn(args.numel, device=dev, generator=torch.Generator(device=dev).manual_seed(g))
             for g in range(2)]

    def round_():
        for c, f in zip(conns, flats):
            c.update_send(f, 1.0)
        got = 0
        for c, f in zip(conns, flats):
            got += c.update_wait_average(f, 1.0)[0] is not None
        return got

    for _ in range(args.warmup):
        round_()
    torch.cuda.synchronize()
    times, averaged = [], 0
    for _ in range(args.rounds):
        t0 = time.perf_counter()
        averaged += round_()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    el = float(np.sum(times))
    out = {
        "what": "two GPU learners gossiping over the reference's TCP protocol (WireConnection), one MI355X, "
                "localhost; fp32, constant 0.5, fetch_probability 1",
        "numel": args.numel,
        "eager_fetch": bool(args.eager),
        "rounds": args.rounds,
        "averagings": averaged,
        "ms_per_round_median": round(1e3 * float(np.median(times)), 2),
        "ms_per_round_min": round(1e3 * float(np.min(times)), 2),
        "averaged_gbs": round(averaged * 3 * args.numel * 4 / el / 1e9, 3),
        "blob_bytes": args.numel * 4,
        "cpu_count": os.cpu_count(),
        "affinity": len(os.sched_getaffinity(0)),
    }
    for c in conns:
        c.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
