#!/usr/bin/env python3
"""Diagnostic: tools/vmm_probe.cpp's fd sharing of hipMemCreate memory, but through the HIP
runtime a torch process loads (torch's bundled libamdhip64), via ctypes, in two spawned
processes -- the runtime the product library runs on in-process.  Usage:
  python tools/vmm_torch_probe.py [chunk MiB] [chunks] [import-mode: value|ptr]"""
import ctypes
import os
import socket
import sys
import time


class Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class Flags(ctypes.Structure):
    _fields_ = [("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class Prop(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("location", Loc),
                ("win32HandleMetaData", ctypes.c_void_p), ("allocFlags", Flags)]


class Access(ctypes.Structure):
    _fields_ = [("location", Loc), ("flags", ctypes.c_int)]


PINNED, POSIX_FD, DEVICE, RW = 1, 1, 1, 3


def hip():
    import torch
    torch.cuda.init()
    with open("/proc/self/maps") as f:
        path = sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})[0]
    lib = ctypes.CDLL(path)
    lib.hipGetErrorString.restype = ctypes.c_char_p
    return lib, path


def ck(lib, rc, what):
    if rc:
        raise RuntimeError("%s: %s" % (what, lib.hipGetErrorString(rc).decode()))


def log(role, msg):
    sys.stderr.write("[%s] %s\n" % (role, msg))
    sys.stderr.flush()


def run(role, address, chunk, k, mode):
    lib, path = hip()
    v = ctypes.c_int()
    lib.hipRuntimeGetVersion(ctypes.byref(v))
    log(role, "runtime %s (%d)" % (path, v.value))
    prop = Prop(PINNED, POSIX_FD, Loc(DEVICE, 0), None, Flags(0, 0, 0))
    acc = Access(Loc(DEVICE, 0), RW)
    va = ctypes.c_void_p()
    ck(lib, lib.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(chunk * k), ctypes.c_size_t(2 << 20), None,
                                     ctypes.c_ulonglong(0)), "reserve")
    if role == "exporter":
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        srv.bind(address)
        srv.listen(1)
        fds = []
        for i in range(k):
            h = ctypes.c_ulonglong()
            ck(lib, lib.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(chunk), ctypes.byref(prop), ctypes.c_ulonglong(0)),
               "create")
            ck(lib, lib.hipMemMap(ctypes.c_void_p(va.value + i * chunk), ctypes.c_size_t(chunk), ctypes.c_size_t(0), h,
                                  ctypes.c_ulonglong(0)), "map")
            fd = ctypes.c_int(-1)
            ck(lib, lib.hipMemExportToShareableHandle(ctypes.byref(fd), h, POSIX_FD, ctypes.c_ulonglong(0)), "export")
            fds.append(fd.value)
        ck(lib, lib.hipMemSetAccess(va, ctypes.c_size_t(chunk * k), ctypes.byref(acc), ctypes.c_size_t(1)), "access")
        for i in range(k):
            ck(lib, lib.hipMemsetD32(ctypes.c_void_p(va.value + i * chunk), ctypes.c_uint(0x11111111 * (i + 1)),
                                     ctypes.c_size_t(chunk // 4)), "memset")
        ck(lib, lib.hipDeviceSynchronize(), "sync")
        log(role, "exported %d fds %s" % (k, fds))
        c, _ = srv.accept()
        socket.send_fds(c, [b"x"], fds)
        c.recv(1)                     # the importer's done byte
        c.close()
        log(role, "importer done")
        return 0
    time.sleep(1.0)
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(address)
    _, fds, _, _ = socket.recv_fds(s, 16, k)
    log(role, "received fds %s" % fds)
    for i, fd in enumerate(fds):
        h = ctypes.c_ulonglong()
        log(role, "importing chunk %d (%s)" % (i, mode))
        if mode == "ptr":
            fdv = ctypes.c_int(fd)
            rc = lib.hipMemImportFromShareableHandle(ctypes.byref(h), ctypes.byref(fdv), POSIX_FD)
        else:
            rc = lib.hipMemImportFromShareableHandle(ctypes.byref(h), ctypes.c_void_p(fd), POSIX_FD)
        ck(lib, rc, "import")
        ck(lib, lib.hipMemMap(ctypes.c_void_p(va.value + i * chunk), ctypes.c_size_t(chunk), ctypes.c_size_t(0), h,
                              ctypes.c_ulonglong(0)), "map")
        log(role, "chunk %d mapped" % i)
    ck(lib, lib.hipMemSetAccess(va, ctypes.c_size_t(chunk * k), ctypes.byref(acc), ctypes.c_size_t(1)), "access")
    out = (ctypes.c_uint * 16)()
    bad = 0
    for i in range(1, k):
        ck(lib, lib.hipMemcpy(out, ctypes.c_void_p(va.value + i * chunk - 32), ctypes.c_size_t(64), 2), "d2h")
        bad += sum(out[j] != (0x11111111 * ((i - 1 if j < 8 else i) + 1)) & 0xFFFFFFFF for j in range(16))
    log(role, "%d boundaries, %d bad words" % (k - 1, bad))
    s.send(b"d")
    s.close()
    return 1 if bad else 0


def main():
    import torch.multiprocessing as mp
    chunk = int(float(sys.argv[1]) * (1 << 20)) if len(sys.argv) > 1 else 2 << 20
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    mode = sys.argv[3] if len(sys.argv) > 3 else "value"
    address = "\0dpwa-vmm-probe-%d" % os.getpid()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=run, args=(role, address, chunk, k, mode)) for role in ("exporter", "importer")]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    print("exit codes", [p.exitcode for p in ps])
    sys.exit(0 if all(p.exitcode == 0 for p in ps) else 1)


if __name__ == "__main__":
    main()
