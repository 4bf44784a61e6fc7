#!/usr/bin/env python3
"""Diagnostic: two ranks on one GPU bind a DistGroup connection over IPC at a given size and
run rounds, logging (to stderr, with a device sync) after every stage.  Usage:
  python tools/ipc_probe.py --numel 1000000000 --dtype bf16 --pull relay:128 --rounds 2"""
import argparse
import os
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, cfg, args):
    t0 = time.perf_counter()

    def log(msg):
        sys.stderr.write("[probe r%d +%.2fs] %s\n" % (rank, time.perf_counter() - t0, msg))
        sys.stderr.flush()
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dpwa_amd import DpwaConnection
    conn = DpwaConnection("r%d" % rank, cfg, seed=500 + rank, pull=args.pull, group="lockstep")
    flat = torch.zeros(args.numel, dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float32, device=dev)
    torch.cuda.synchronize()
    log("allocated %d" % args.numel)
    conn._bind(flat)
    torch.cuda.synchronize()
    log("bound (IPC exchanged)")
    for r in range(args.rounds):
        conn.update_send(flat, 1.0)
        torch.cuda.synchronize()
        log("round %d update_send" % r)
        payload, _ = conn.update_wait_average(flat, 1.0)
        torch.cuda.synchronize()
        log("round %d averaged with %s" % (r, payload.peer if payload is not None else "-"))
    dist.barrier()
    conn.close()
    dist.destroy_process_group()
    log("done")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=int, default=1_000_000)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--pull", default="copy")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    from dpwa_amd.launch import write_config
    cfg = write_config(os.path.join(tempfile.mkdtemp(), "probe.yaml"), ["r0", "r1"])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(2, port, cfg, args), nprocs=2, join=True)


if __name__ == "__main__":
    main()
