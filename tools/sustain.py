#!/usr/bin/env python3
"""How the N=1 resident pair loop's round time evolves under sustained load (tooling, not part of
the product): us/round in consecutive ~50 ms windows over SECONDS of continuous rounds, then an
idle pause, then more windows -- does the chip slow down as it keeps streaming (power or thermal
limits) and recover when idle?  Samples rocm-smi's clocks/power before, during and after when it
is available (read-only)."""
import os
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from dpwa_amd import DpwaConnection  # noqa: E402
from dpwa_amd.group import LocalGroup  # noqa: E402

N = bench.RESNET18_NUMEL
DEV = torch.device("cuda", 0)


def smi(tag):
    try:
        out = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--showtemp"], capture_output=True,
                             text=True, timeout=20).stdout
    except Exception as e:      # noqa: BLE001
        out = "rocm-smi unavailable: %s" % e
    keep = [ln.strip() for ln in out.splitlines() if any(k in ln for k in ("Power", "mclk", "sclk", "fclk",
                                                                             "Temperature", "socclk"))]
    print("[%s] %s" % (tag, " | ".join(keep)), flush=True)


def main():
    seconds = float(os.environ.get("SUSTAIN_S", "8"))
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

    def rounds(k):
        for _ in range(k):
            for c, f in zip(conns, flats):
                c.update_send(f, 1.0, reuse_snapshot=True)
            DpwaConnection.update_wait_average_many(conns, flats, [1.0, 1.0])
            flats[:] = [c.parameters for c in conns]

    def series(tag, secs):
        out = []
        t_end = time.perf_counter() + secs
        while time.perf_counter() < t_end:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rounds(1500)
            torch.cuda.synchronize()
            out.append(1e6 * (time.perf_counter() - t0) / 1500)
        print("%s us/round per ~45 ms window: %s" % (tag, " ".join("%.1f" % x for x in out)), flush=True)

    rounds(200)
    torch.cuda.synchronize()
    smi("idle, before")
    time.sleep(2.0)
    th = threading.Timer(seconds / 2, smi, args=("under load",))
    th.start()
    series("sustained %.0f s" % seconds, seconds)
    th.join()
    smi("right after")
    for pause in (0.5, 2.0, 5.0):
        time.sleep(pause)
        series("after %.1f s idle" % pause, 1.0)
    for c in conns:
        c.close()


if __name__ == "__main__":
    main()
