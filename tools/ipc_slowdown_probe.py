#!/usr/bin/env python3
"""Diagnostic: does mapping another process's device memory (hipIpcOpenMemHandle) slow this
process's kernels?  Two ranks on one GPU time a conv workload before the exchange, after
each exports a buffer and opens the other's, and after closing; optional --vmm uses the
fd-shared hipMemCreate path (the product's DPWA_VMM=1) through DpwaConnection instead."""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bench(torch, dev, reps=60):
    """ms per iteration of a conv and a GEMM (the training step's two kernel families)."""
    x = torch.randn(128, 64, 32, 32, device=dev)
    conv = torch.nn.Conv2d(64, 64, 3, padding=1).to(dev)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    with torch.no_grad():
        for _ in range(5):
            conv(x)
            a @ a
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            conv(x)
            a @ a
        torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / reps


def worker(rank, port, mode):
    import ctypes

    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {"before": bench(torch, dev)}
    dist.barrier()
    if mode == "none":                 # control: same barriers and benchmarks, no mapping
        dist.barrier()
        out["mapped"] = bench(torch, dev)
        dist.barrier()
        dist.barrier()
        out["closed"] = bench(torch, dev)
    elif mode.startswith("hipipc"):
        one_way = mode == "hipipc-oneway"          # rank 0 only exports, rank 1 only opens
        with open("/proc/self/maps") as f:
            path = sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})[0]
        lib = ctypes.CDLL(path)

        class H(ctypes.Structure):
            _fields_ = [("r", ctypes.c_char * 64)]
        lib.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), H, ctypes.c_uint]
        buf = torch.empty(100 << 20, dtype=torch.uint8, device=dev)
        h = H()
        assert lib.hipIpcGetMemHandle(ctypes.byref(h), ctypes.c_void_p(buf.data_ptr())) == 0
        hs = [None, None]
        dist.all_gather_object(hs, ctypes.string_at(ctypes.addressof(h), 64))
        other = H.from_buffer_copy(hs[1 - rank])
        p = ctypes.c_void_p()
        opens = not one_way or rank == 1
        if opens:
            assert lib.hipIpcOpenMemHandle(ctypes.byref(p), other, 1) == 0
        dist.barrier()
        out["mapped"] = bench(torch, dev)
        dist.barrier()
        if opens:
            lib.hipIpcCloseMemHandle(p)
        dist.barrier()
        out["closed"] = bench(torch, dev)
    else:
        from dpwa_amd import DpwaConnection
        from dpwa_amd.launch import write_config
        cfg = os.path.join("/tmp", "slow_%d.yaml" % port)
        if rank == 0:
            write_config(cfg, ["r0", "r1"])
        dist.barrier()
        conn = DpwaConnection("r%d" % rank, cfg, seed=rank, group=mode)
        flat = torch.zeros(11_173_962, device=dev)
        conn.update_send(flat, 1.0)                     # binds: exports and maps the slots
        torch.cuda.synchronize()
        dist.barrier()
        out["mapped"] = bench(torch, dev)
        dist.barrier()
        conn.close()
        dist.barrier()
        out["closed"] = bench(torch, dev)
    print("rank %d %s %s" % (rank, mode, {k: round(v, 3) for k, v in out.items()}), flush=True)
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    mode = sys.argv[1] if len(sys.argv) > 1 else "hipipc"      # hipipc | lockstep | async
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(port, mode), nprocs=2, join=True)


if __name__ == "__main__":
    main()
