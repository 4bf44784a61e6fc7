#!/usr/bin/env python3
"""The drop-in adapter's round on its own, for traces: DpwaPyTorchAdapter over one parameter of
--numel elements, configs[1]'s self-peer YAML (bench.write_config), its defaults (write-through,
reuse guard on; --no-guard, --resident to change them), update_send -> update_wait for --rounds
rounds after --warmup.  Run it under `DPWA_ROCTX=1 rocprofv3 --marker-trace --kernel-trace` and
feed the output to tools/marker_gaps.py.  Prints one JSON line (ms per round, wall clock)."""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from dpwa_amd import DpwaPyTorchAdapter, _lib  # noqa: E402
from dpwa_amd.group import LocalGroup  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=int, default=bench.RESNET18_NUMEL)
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32")
    ap.add_argument("--rounds", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--no-guard", action="store_true")
    ap.add_argument("--resident", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dtype = torch.float32 if a.dtype == "f32" else torch.bfloat16
    tmp = tempfile.mkdtemp(prefix="dpwa_adapter_")
    cfg = os.path.join(tmp, "self.yaml")
    bench.write_config(cfg, ["a1"], "constant", self_peer=True, base_port=45600)
    net = torch.nn.Module()
    g = torch.Generator(device=dev).manual_seed(0)
    net.register_parameter("w", torch.nn.Parameter(torch.randn(a.numel, device=dev, generator=g).to(dtype)))
    ad = DpwaPyTorchAdapter(net, "a1", cfg, seed=3000, group=LocalGroup(), reuse_guard=not a.no_guard,
                            resident=a.resident)
    for _ in range(a.warmup):
        ad.update_send(1.0)
        ad.update_wait(1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        ad.update_send(1.0)
        ad.update_wait(1.0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"numel": a.numel, "dtype": a.dtype, "rounds": a.rounds, "ms_per_round": round(1e3 * el / a.rounds, 4),
                      "reuse_guard": not a.no_guard, "resident": a.resident, "trace": _lib.TRACE,
                      "guard_hits": ad.window_guard_hits if a.resident else ad.reuse_guard_hits}))
    ad.connection.close()


if __name__ == "__main__":
    main()
