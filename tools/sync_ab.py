#!/usr/bin/env python3
"""How much of a short timed region is the host noticing the GPU has finished?  configs[1]'s
self-peer connection loop (bench.py's timed rounds), K rounds per timed region, the region
closed by (a) torch.cuda.synchronize() alone or (b) a spin on an event recorded after the last
round, then torch.cuda.synchronize(); A/B interleaved over many regions.  Also the same K rounds
timed by events on the stream (the GPU's own view).  Prints one JSON line."""
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from dpwa_amd import DpwaConnection  # noqa: E402
from dpwa_amd.group import LocalGroup  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    regions = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda", 0)
    tmp = tempfile.mkdtemp(prefix="dpwa_sync_")
    cfg = os.path.join(tmp, "self.yaml")
    bench.write_config(cfg, ["w1"], "constant", self_peer=True, base_port=45700)
    flat = torch.randn(bench.RESNET18_NUMEL, device=dev)
    conn = DpwaConnection("w1", cfg, seed=1000, group=LocalGroup())

    def rounds(k):
        for _ in range(k):
            conn.update_send(flat, 1.0, reuse_snapshot=True)
            conn.update_wait_average(flat, 1.0, write_through=True)

    rounds(200)
    torch.cuda.synchronize()
    out = {"sync": [], "spin": [], "events": []}
    stream = torch.cuda.current_stream(dev)
    for i in range(regions):
        for mode in (("sync", "spin") if i % 2 == 0 else ("spin", "sync")):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            rounds(K)
            e1.record(stream)
            if mode == "spin":
                while not e1.query():
                    pass
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            out[mode].append(1e6 * el / K)
            out["events"].append(1e3 * e0.elapsed_time(e1) / K)
    res = {"rounds_per_region": K, "regions": regions,
           "us_per_round_median": {k: round(statistics.median(v), 3) for k, v in out.items()},
           "us_per_round_mean": {k: round(statistics.mean(v), 3) for k, v in out.items()}}
    print(json.dumps(res))
    conn.close()


if __name__ == "__main__":
    main()
