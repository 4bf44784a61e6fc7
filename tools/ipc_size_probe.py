#!/usr/bin/env python3
"""Diagnostic: the largest hipMalloc allocation that two processes on one GPU can share with
hipIpcGetMemHandle / hipIpcOpenMemHandle.  Each size is exported by rank 0 and opened by
rank 1, with a log line (stderr) around every HIP call.  Usage:
  python tools/ipc_size_probe.py 1 2 3 4 5        (sizes in GiB)"""
import ctypes
import os
import socket
import sys
import time


def hip():
    """The HIP runtime torch has loaded (same file -> same handle; never a second runtime)."""
    import torch
    torch.cuda.init()
    with open("/proc/self/maps") as f:
        paths = sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})
    lib = ctypes.CDLL(paths[0])
    lib.hipGetErrorString.restype = ctypes.c_char_p
    lib.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    return lib


class Handle(ctypes.Structure):           # hipIpcMemHandle_t, passed by value
    _fields_ = [("reserved", ctypes.c_char * 64)]


def worker(rank, port, sizes):
    t0 = time.perf_counter()

    def log(msg):
        sys.stderr.write("[ipc r%d +%.2fs] %s\n" % (rank, time.perf_counter() - t0, msg))
        sys.stderr.flush()
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.cuda.set_device(0)
    lib = hip()
    for gib in sizes:
        nbytes = int(gib * (1 << 30))
        ptr = ctypes.c_void_p()
        handle = ctypes.create_string_buffer(64)
        if rank == 0:
            rc = lib.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(nbytes))
            log("%.2f GiB hipMalloc rc=%d" % (gib, rc))
            rc = lib.hipIpcGetMemHandle(handle, ptr)
            log("%.2f GiB hipIpcGetMemHandle rc=%d" % (gib, rc))
        blob = [handle.raw if rank == 0 else None]
        dist.broadcast_object_list(blob, src=0)
        if rank == 1:
            h = Handle.from_buffer_copy(blob[0])
            opened = ctypes.c_void_p()
            log("%.2f GiB hipIpcOpenMemHandle ..." % gib)
            rc = lib.hipIpcOpenMemHandle(ctypes.byref(opened), h, ctypes.c_uint(1))
            log("%.2f GiB hipIpcOpenMemHandle rc=%d (%s)" % (gib, rc, lib.hipGetErrorString(rc).decode()))
            if rc == 0:
                lib.hipIpcCloseMemHandle(opened)
        dist.barrier()
        if rank == 0:
            lib.hipFree(ptr)
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    sizes = [float(x) for x in sys.argv[1:]] or [1, 2, 3, 4, 5]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(port, sizes), nprocs=2, join=True)


if __name__ == "__main__":
    main()
