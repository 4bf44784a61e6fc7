#!/usr/bin/env python3
"""Host cost of one gossip round: configs[1]'s self-peer connection loop (bench.py's timed
round: update_send(reuse_snapshot) + update_wait_average(write_through)) and the adapter's round,
on a parameter small enough (--numel, default 4,096) that the device never holds the host back,
so wall time per round = the host's issue time.  Also each call alone (perf_counter around it).
Prints one JSON line."""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter  # noqa: E402
from dpwa_amd.group import LocalGroup  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    tmp = tempfile.mkdtemp(prefix="dpwa_host_")
    cfg = os.path.join(tmp, "self.yaml")
    bench.write_config(cfg, ["w1"], "constant", self_peer=True, base_port=45800)
    flat = torch.randn(a.numel, device=dev)
    conn = DpwaConnection("w1", cfg, seed=1000, group=LocalGroup())
    res = {"numel": a.numel, "rounds": a.rounds}

    def conn_round():
        conn.update_send(flat, 1.0, reuse_snapshot=True)
        conn.update_wait_average(flat, 1.0, write_through=True)

    for _ in range(200):
        conn_round()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        conn_round()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    res["conn_issue_us"] = round(1e6 * (t1 - t0) / a.rounds, 3)
    send, wait = [], []
    for _ in range(a.rounds):
        s0 = time.perf_counter()
        conn.update_send(flat, 1.0, reuse_snapshot=True)
        s1 = time.perf_counter()
        conn.update_wait_average(flat, 1.0, write_through=True)
        s2 = time.perf_counter()
        send.append(s1 - s0)
        wait.append(s2 - s1)
    torch.cuda.synchronize()
    res["conn_update_send_us_median"] = round(1e6 * statistics.median(send), 3)
    res["conn_update_wait_average_us_median"] = round(1e6 * statistics.median(wait), 3)
    conn.close()

    cfg2 = os.path.join(tmp, "adapter.yaml")
    bench.write_config(cfg2, ["a1"], "constant", self_peer=True, base_port=45850)
    for guard in (True, False):
        net = torch.nn.Module()
        net.register_parameter("w", torch.nn.Parameter(torch.randn(a.numel, device=dev)))
        ad = DpwaPyTorchAdapter(net, "a1", cfg2, seed=3000, group=LocalGroup(), reuse_guard=guard)
        for _ in range(200):
            ad.update_send(1.0)
            ad.update_wait(1.0)
        torch.cuda.synchronize()
        send, wait = [], []
        t0 = time.perf_counter()
        for _ in range(a.rounds):
            s0 = time.perf_counter()
            ad.update_send(1.0)
            s1 = time.perf_counter()
            ad.update_wait(1.0)
            s2 = time.perf_counter()
            send.append(s1 - s0)
            wait.append(s2 - s1)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        key = "adapter_guard" if guard else "adapter_noguard"
        res[key + "_issue_us"] = round(1e6 * (t1 - t0) / a.rounds, 3)
        res[key + "_update_send_us_median"] = round(1e6 * statistics.median(send), 3)
        res[key + "_update_wait_us_median"] = round(1e6 * statistics.median(wait), 3)
        ad._conn.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
