#!/usr/bin/env python3
"""Times the REFERENCE's own CPU gossip round (zenghanfu/dpwa, imported read-only from
/root/reference) in the build container: two learner processes on localhost, real
RxThread/TxThread sockets, pickle framing and the adapter's torch-CPU lerp -- exactly the
path BASELINE.md's CPU rows describe.  The GPU box has no copy of the reference, so this
runs here and its result is committed as profiles/reference_cpu_r01.json.

Only runtime patch: yaml.load gets a SafeLoader (dpwa/dpwa.py:31 fails on PyYAML 6).

Usage: python tools/reference_cpu_timing.py [--numel N ...] [--rounds K] [--out FILE]
"""
import argparse
import functools
import json
import multiprocessing as mp
import os
import platform
import sys
import tempfile
import time

REF = os.environ.get("DPWA_REFERENCE", "/root/reference")


def learner(name, cfg, numel, rounds, q, threads, core=None):
    if core is not None:
        os.sched_setaffinity(0, {core})      # taskset -c <core> (prepare.py:31)
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import logging
    logging.disable(logging.CRITICAL)
    import torch
    torch.set_num_threads(threads)
    import yaml
    yaml.load = functools.partial(yaml.load, Loader=yaml.SafeLoader)
    from dpwa.adapters.pytorch import DpwaPyTorchAdapter

    class Flat(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.randn(numel))

    net = Flat()
    import random
    random.seed(1 if name == "w1" else 2)
    conn = DpwaPyTorchAdapter(net, name, cfg)
    time.sleep(1.0)                      # let both servers listen
    conn.update_send(1.0)                # warm-up round (connects)
    conn.update_wait(1.0)
    times = []
    split = {"send": 0.0, "wait": 0.0}
    for _ in range(rounds):
        t0 = time.perf_counter()
        conn.update_send(1.0)
        t1 = time.perf_counter()
        conn.update_wait(1.0)
        t2 = time.perf_counter()
        times.append(t2 - t0)
        split["send"] += t1 - t0
        split["wait"] += t2 - t1
    q.put((name, times, split))
    time.sleep(2.0)                      # keep serving until the other side is done
    os._exit(0)                          # reference threads never exit (conn.py:170-172)


def run(numel, rounds, threads, pin=False):
    with tempfile.TemporaryDirectory() as tmp:
        cfg = os.path.join(tmp, "c.yaml")
        base = 46100 + (numel % 500)
        with open(cfg, "w") as f:
            f.write("- nodes:\n  - {name: w1, host: localhost, port: %d}\n  - {name: w2, host: localhost, port: %d}\n"
                    "- fetch_probability: 1\n- timeout_ms: 600000\n- interpolation: constant\n"
                    "- divergence_threshold: 0\n- constant: { value: 0.5 }\n- clock: 0\n- loss: 0\n" % (base, base + 1))
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        cores = sorted(os.sched_getaffinity(0))[:2] if pin else [None, None]
        ps = [ctx.Process(target=learner, args=(n, cfg, numel, rounds, q, threads, c))
              for n, c in zip(("w1", "w2"), cores)]
        for p in ps:
            p.start()
        res = {}
        for _ in ps:
            name, times, split = q.get(timeout=3600)
            res[name] = (times, split)
        for p in ps:
            p.join(timeout=30)
    times = sorted(res["w1"][0] + res["w2"][0])
    med = times[len(times) // 2]
    return {"numel": numel, "rounds_per_learner": rounds, "median_round_s": med,
            "averaged_GBps": 3 * numel * 4 / med / 1e9,
            "averaged_GBps_both_learners": 2 * 3 * numel * 4 / med / 1e9,
            "pinned_cores": cores,
            "mean_send_s": (res["w1"][1]["send"] + res["w2"][1]["send"]) / (2 * rounds),
            "mean_wait_s": (res["w1"][1]["wait"] + res["w2"][1]["wait"]) / (2 * rounds)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=int, nargs="+", default=[11_173_962, 100_000_000])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--threads", type=int, default=1, help="torch threads per learner (prepare.py:31 uses 1)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--pin", action="store_true", help="pin each learner to its own core (taskset, prepare.py:31)")
    ap.add_argument("--port-seconds", type=float, default=0.0,
                    help="also time oracle/ref_round.py (the restatement bench.py runs on the GPU box) at the same "
                         "sizes, and report the port/reference round-time ratio")
    args = ap.parse_args()
    rows = [run(n, args.rounds if n < 50_000_000 else max(3, args.rounds // 2), args.threads, args.pin)
            for n in args.numel]
    out = {"what": "reference dpwa CPU round (update_send + update_wait) between 2 localhost learners: "
                   "TCP + pickle + torch-CPU lerp, fp32, constant 0.5, fetch_probability 1",
           "source": "dpwa/adapters/pytorch.py:42-68, dpwa/dpwa.py:104-156, dpwa/conn.py:98-329",
           "host": {"cpus": os.cpu_count(), "machine": platform.processor() or platform.machine(),
                    "torch_threads_per_learner": args.threads},
           "rows": rows}
    if args.port_seconds > 0:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import ref_round
        ports = [ref_round.run(r["numel"], args.port_seconds, min_rounds=3) for r in rows]
        out["port_rows"] = ports
        out["port_vs_reference"] = [
            {"numel": r["numel"], "reference_median_round_ms": round(1e3 * r["median_round_s"], 2),
             "port_median_round_ms": p["median_round_ms"],
             "port_over_reference_rate": round(1e3 * r["median_round_s"] / p["median_round_ms"], 3)}
            for r, p in zip(rows, ports)]
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
