"""The reference's CPU gossip round, restated for timing on the GPU box -- TEST/BASELINE
INFRASTRUCTURE ONLY (see oracle/__init__.py): ``bench.py``'s ``cpu_baseline`` leg runs it.

/root/reference does not exist on the GPU box, so the reference's own CPU path (timed in the
build container by tools/reference_cpu_timing.py -> profiles/reference_cpu_r01.json) is
restated here -- no reference code is imported or copied -- and timed on the box's host
cores in the same run as the GPU path (CPU-baseline plan item 1).  One learner
per process, as prepare.py:28-36 launches them; each has a server thread (RxThread) and runs
its rounds free-running, as the reference does:

  update_send   dpwa/adapters/pytorch.py:49-53   every tensor -> raw fp32 bytes in a dict,
                                                  pickle.dumps(dict)
                dpwa/dpwa.py:111-116, conn.py:73-79  clock += 1, publish (state, blob) under
                                                  the server's lock
  fetch         conn.py:286-302 -> messaging.py:76-94 / 36-73
                                                  10-byte request; the server replies with the
                                                  <HLL header + pickle(state) + blob in 8 MiB
                                                  sends under its lock (conn.py:109-110); the
                                                  client accumulates ``blob += chunk`` (the
                                                  reference's receive loop, messaging.py:49-56)
  update_wait   dpwa/dpwa.py:139-155              factor (constant 0.5 here) and clock
                dpwa/adapters/pytorch.py:64-68    pickle.loads, then per tensor
                                                  f32(f32(a*t) + f32(b*p)) (oracle.lerp.lerp_f32)

The parameter set is ResNet-18's 62 tensors (11,173,962 fp32; examples/pytorch-cifar/
models/resnet.py:102-103), or one flat tensor of any other size.
"""
import multiprocessing as mp
import os
import pickle
import socket
import struct
import threading
import time

import numpy as np

from .lerp import lerp_f32

HEADER_FMT = "<HLL"            # messaging.py:16
HEADER_LEN = 10                # messaging.py:15
CHUNK_SIZE = 8 * (1024 ** 2)   # messaging.py:17
FETCH = 1                      # conn.py:34 MESSAGE_TYPE_FETCH_PARAMETERS


def resnet18_shapes(num_classes=10):
    """Parameter shapes of ResNet18 (models/resnet.py:102-103, BasicBlock), in
    named_parameters() order: 62 tensors, 11,173,962 elements."""
    shapes = [(64, 3, 3, 3), (64,), (64,)]
    cin = 64
    for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
        for b in range(2):
            s = stride if b == 0 else 1
            shapes += [(cout, cin, 3, 3), (cout,), (cout,), (cout, cout, 3, 3), (cout,), (cout,)]
            if s != 1 or cin != cout:
                shapes += [(cout, cin, 1, 1), (cout,), (cout,)]
            cin = cout
    shapes += [(num_classes, 512), (num_classes,)]
    return shapes


def _sizes(numel):
    shapes = resnet18_shapes()
    if sum(int(np.prod(s)) for s in shapes) == numel:
        return [int(np.prod(s)) for s in shapes]
    return [numel]


def send_message(sock, mtype, message=None, payload=None):
    """messaging.py:76-94."""
    raw = b"" if message is None else pickle.dumps(message)
    payload = b"" if payload is None else payload
    blob = struct.pack(HEADER_FMT, mtype, len(raw), len(payload)) + raw + payload
    count = 0
    while count < len(blob):
        sent = sock.send(blob[count:count + CHUNK_SIZE])
        if sent == 0:
            raise ConnectionError("send() failed")
        count += sent


def recv_message(sock):
    """messaging.py:36-73 (including its ``blob += chunk`` accumulation).  The frames come
    from this module's own server thread in the same benchmark, never from the network."""
    first = sock.recv(CHUNK_SIZE + HEADER_LEN)
    if not first:
        raise ConnectionError("recv() failed")
    mtype, mlen, plen = struct.unpack(HEADER_FMT, first[:HEADER_LEN])
    total = mlen + plen
    blob = first[HEADER_LEN:]
    count = len(blob)
    while count < total:
        chunk = sock.recv(CHUNK_SIZE)
        if not chunk:
            raise ConnectionError("recv() failed")
        blob += chunk
        count += len(chunk)
    message = pickle.loads(blob[:mlen]) if mlen else None
    payload = blob[mlen:] if plen else None
    return mtype, message, payload


class _Server(threading.Thread):
    """RxThread (conn.py:51-168) for one client: serves the latest (state, payload)."""

    def __init__(self):
        super().__init__(daemon=True)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(10)
        self.port = self.sock.getsockname()[1]
        self.lock = threading.Lock()
        self.state = None
        self.payload = None

    def publish(self, state, payload):
        with self.lock:
            self.state, self.payload = dict(state), payload

    def run(self):
        conn, _ = self.sock.accept()
        conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        try:
            while True:
                mtype, _, _ = recv_message(conn)
                if mtype != FETCH:
                    break
                if self.payload is None:
                    send_message(conn, FETCH)
                else:
                    with self.lock:
                        send_message(conn, FETCH, self.state, self.payload)
        except (ConnectionError, OSError):
            pass
        conn.close()


def _learner(idx, numel, seconds, min_rounds, core, port_q, peer_q, start, out_q, finish):
    if core is not None:
        os.sched_setaffinity(0, {core})        # taskset -c <core> (prepare.py:31)
    rng = np.random.default_rng(idx)
    params = {"p%d" % i: rng.standard_normal(k).astype(np.float32) for i, k in enumerate(_sizes(numel))}
    server = _Server()
    server.start()
    port_q.put((idx, server.port))
    client = socket.create_connection(("127.0.0.1", peer_q.get()))
    client.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    clock, factor, loss = 0.0, 0.5, 1.0
    rounds, busy = 0, 0.0
    phases = []          # per averaged round: (pickle, fetch, unpickle, lerp) seconds
    start.wait()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds or rounds < min_rounds:
        t = time.perf_counter()
        blob = pickle.dumps({k: bytes(v) for k, v in params.items()})      # update_send
        clock += 1
        server.publish({"clock": clock, "loss": loss}, blob)
        t1 = time.perf_counter()
        send_message(client, FETCH)                                           # fetch
        _, state, payload = recv_message(client)
        t2 = time.perf_counter()
        if payload is not None:                                               # update_wait
            clock = factor * state["clock"] + (1 - factor) * clock
            other = pickle.loads(payload)
            t3 = time.perf_counter()
            for k in params:
                params[k] = lerp_f32(params[k], np.frombuffer(other[k], dtype=np.float32), factor)
            t4 = time.perf_counter()
            rounds += 1
            phases.append((t1 - t, t2 - t1, t3 - t2, t4 - t3))
        busy += time.perf_counter() - t
    out_q.put((idx, rounds, busy, time.perf_counter() - t0, phases))
    finish.wait(timeout=3600)   # keep serving (server thread) until the other learner is done too
    client.close()


def _cores():
    """Two distinct cores this process may run on (the learners are pinned one each)."""
    allowed = sorted(os.sched_getaffinity(0))
    return (allowed[0], allowed[1]) if len(allowed) >= 2 else (None, None)


def run(numel=11_173_962, seconds=10.0, min_rounds=0):
    """Two learner processes on localhost, each pinned to its own core, for about `seconds` of
    rounds each (and at least `min_rounds` averagings); returns the cpu_baseline dict:
    aggregate averaged GB/s (3*numel*4 bytes per completed averaging, both learners, over the
    wall time), the mean and median round time and the per-phase split of a round."""
    ctx = mp.get_context("spawn")
    port_q, out_q = ctx.Queue(), ctx.Queue()
    peer_qs = [ctx.Queue(), ctx.Queue()]
    start = ctx.Event()
    finish = ctx.Barrier(2)
    env = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "1"          # one core per learner, as prepare.py:31 pins them
    cores = _cores()
    try:
        procs = [ctx.Process(target=_learner, args=(i, numel, seconds, min_rounds, cores[i], port_q, peer_qs[i],
                                                    start, out_q, finish), daemon=True)
                 for i in range(2)]
        for p in procs:
            p.start()
    finally:
        os.environ.clear()
        os.environ.update(env)
    ports = dict(port_q.get(timeout=300) for _ in procs)
    peer_qs[0].put(ports[1])
    peer_qs[1].put(ports[0])
    start.set()
    res = [out_q.get(timeout=seconds * 30 + 600) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.terminate()
    rounds = sum(r[1] for r in res)
    wall = max(r[3] for r in res)
    phases = np.array([ph for r in res for ph in r[4]]) if rounds else np.zeros((1, 4))
    med = np.median(phases, axis=0) * 1e3
    per_round = phases.sum(axis=1) * 1e3
    return {"value": rounds * 3 * numel * 4 / wall / 1e9, "unit": "GB/s", "cores": 2, "kind": "port",
            "sample": "the reference's CPU round restated (oracle/ref_round.py): 2 learner processes, each pinned to "
                      "one core (taskset -c %s / %s, OMP_NUM_THREADS=1, as prepare.py:31), localhost TCP, pickle + "
                      "<HLL framing + numpy fp32 lerp over %s (%d elements); %d averagings in %.1f s"
                      % (cores[0], cores[1], "ResNet-18's 62 tensors" if len(_sizes(numel)) > 1 else "one flat tensor",
                         numel, rounds, wall),
            "numel": numel,
            "ms_per_round": round(1e3 * sum(r[2] for r in res) / max(1, rounds), 2),
            "median_round_ms": round(float(np.median(per_round)), 2),
            "rounds": rounds,
            "phases_median_ms": {"pickle": round(float(med[0]), 2), "fetch": round(float(med[1]), 2),
                                 "unpickle": round(float(med[2]), 2), "lerp": round(float(med[3]), 2)},
            "phases_note": "per averaged round of one learner: pickle = update_send's bytes() + pickle.dumps + "
                           "publish under the server lock (pytorch.py:49-53, conn.py:73-79); fetch = request + the "
                           "peer's reply over TCP incl. its chunked send and the blob += chunk receive (conn.py:"
                           "297-298, messaging.py:36-94); unpickle = pickle.loads (pytorch.py:64); lerp = per-tensor "
                           "f32(a*t)+f32(b*p) (pytorch.py:66-68)",
            "taskset": [cores[0], cores[1]],
            "cpu_count": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0))}
