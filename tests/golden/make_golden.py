#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE.

Test infrastructure only.  This script runs in the build container, where the
reference (zenghanfu/dpwa) is mounted read-only at /root/reference; it never runs
on the GPU box and nothing in the product imports it.  The reference is imported
unmodified (PYTHONDONTWRITEBYTECODE keeps the tree untouched).  The only runtime
patches are attribute swaps in the imported modules' namespaces:

* ``yaml.load`` gets ``Loader=yaml.SafeLoader``: dpwa/dpwa.py:31 calls it without a
  Loader, which raises TypeError on PyYAML 6.
* ``dpwa.dpwa.RxThread`` -> ``FakeRx``: holds ``(state, payload)`` exactly like
  RxThread.set_current_state (dpwa/conn.py:73-79) but opens no server socket.
* ``dpwa.conn._create_tcp_socket``, ``send_message`` and ``recv_message`` -> in-process
  fakes, so the real ``TxThread`` selection/retry loop (dpwa/conn.py:224-317) runs
  against scripted peers instead of TCP.
* ``dpwa.dpwa.random`` / ``dpwa.conn.random`` -> ``RngDispatch``: per-learner
  ``random.Random`` instances, so G learners driven from one process draw exactly
  the streams that G separate processes, each after ``random.seed(seed_g)``, draw.

Outputs (all small; see tests/golden/README.md):
  lerp_f32.npz          adapter update_wait lerp (dpwa/adapters/pytorch.py:55-68)
  lerp_bf16.npz         torch-eager bf16 form (reference has no bf16 path: pytorch.py:11-14)
  policy.json           factor / clock / Bernoulli traces (dpwa/dpwa.py:101-156, interpolation.py)
  peer_select.json      TxThread peer choice + flow control under scripted faults (conn.py:224-317)
  peer_add.json         the same with removed peers put back by add_peer (dpwa.py:95-96, conn.py:208-213)
  gossip.npz/.json      lock-step G-learner gossip through the real adapter + connection + TxThread
  gossip_step_after_wait.npz/.json   the same with the step after update_wait (the resident order)
  gossip_self.npz/.json one learner whose peer is its own RxThread (a node entry at its own address)
  wire.json             <HLL + pickle frames (dpwa/messaging.py:24-94)
  config.json           YAML parsing (dpwa/dpwa.py:29-93)

Usage:  python tests/golden/make_golden.py   (from the repo root)
"""
import copy
import functools
import json
import math
import os
import random
import socket
import sys
import tempfile
import threading

import numpy as np

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REF = os.environ.get("DPWA_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

import torch  # noqa: E402
import yaml  # noqa: E402

yaml.load = functools.partial(yaml.load, Loader=yaml.SafeLoader)

import dpwa.conn as rconn  # noqa: E402
import dpwa.dpwa as rdpwa  # noqa: E402
import dpwa.messaging as rmsg  # noqa: E402
from dpwa.adapters.pytorch import DpwaPyTorchAdapter  # noqa: E402

import logging  # noqa: E402

logging.disable(logging.CRITICAL)

OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------
# Runtime fakes
# ----------------------------------------------------------------------------
class RngDispatch:
    """Routes ``random.random`` / ``random.randint`` to the active learner's stream.

    The learner is looked up by thread: the driver thread sets ``current`` before
    calling into a learner; each learner's TxThread is registered by ident.
    """

    def __init__(self):
        self.rngs = {}
        self.by_thread = {}
        self.local = threading.local()

    def set_current(self, key):
        self.local.key = key

    def _rng(self):
        key = self.by_thread.get(threading.get_ident())
        if key is None:
            key = self.local.key
        return self.rngs[key]

    def random(self):
        return self._rng().random()

    def randint(self, a, b):
        return self._rng().randint(a, b)


RNG = RngDispatch()
rdpwa.random = RNG
rconn.random = RNG


class FakeRx:
    """Stand-in for RxThread: stores the published (state, payload)."""

    registry = {}

    def __init__(self, host, port, timeout_ms):
        self.addr = (host, port)
        self.lock = threading.Lock()
        self.have_state = False
        self.state = None
        self.payload = None
        FakeRx.registry[self.addr] = self

    def set_current_state(self, state, payload):
        with self.lock:
            self.state = copy.deepcopy(state)
            self.payload = copy.deepcopy(payload)
            self.have_state = True

    def start(self):
        pass


rdpwa.RxThread = FakeRx


class Env:
    """Decides connect/request outcomes for the fake sockets and logs attempts."""

    def __init__(self):
        self.logs = {}         # learner name -> attempt dicts of its current round
        self.connect_fn = lambda peer: "ok"
        self.request_fn = lambda peer: "payload"
        self.reply_fn = lambda peer: ({"clock": 1, "loss": 1.0}, b"x")
        self.gate = None       # threading.Event the request waits on (lock-step gossip)


ENV = Env()
ADDR2NAME = {}


class FakeSock:
    def __init__(self):
        self.peer = None
        self.owner = RNG.by_thread[threading.get_ident()]   # the learner whose TxThread dials

    def settimeout(self, t):
        pass

    def connect(self, addr):
        self.peer = ADDR2NAME[addr]
        out = ENV.connect_fn(self.peer)
        ENV.logs[self.owner].append({"peer": self.peer, "connect": out, "request": None})
        if out == "refused":
            raise ConnectionRefusedError("scripted refusal")
        if out == "error":
            raise OSError("scripted unrecoverable connect error")

    def close(self):
        pass

    def fileno(self):
        return 1000


def fake_create_tcp_socket():
    return FakeSock()


def fake_send_message(sock, message_type, message=None, payload=None):
    assert message_type == rconn.MESSAGE_TYPE_FETCH_PARAMETERS
    sock.pending = True


def fake_recv_message(sock):
    if ENV.gate is not None:
        ENV.gate.wait()
    log = ENV.logs[sock.owner]
    if not log or log[-1]["peer"] != sock.peer or log[-1]["request"] is not None:
        log.append({"peer": sock.peer, "connect": None, "request": None})
    out = ENV.request_fn(sock.peer)
    log[-1]["request"] = out
    if out == "payload":
        state, payload = ENV.reply_fn(sock.peer)
        return rconn.MESSAGE_TYPE_FETCH_PARAMETERS, state, payload
    if out == "empty":
        return rconn.MESSAGE_TYPE_FETCH_PARAMETERS, None, None
    if out == "timeout":
        raise socket.timeout("scripted timeout")
    raise RuntimeError("scripted request error")


rconn._create_tcp_socket = fake_create_tcp_socket
rconn.send_message = fake_send_message
rconn.recv_message = fake_recv_message


def write_config(path, nodes, fetch_p, interp, thr, extra=None, timeout_ms=2500):
    lines = ["---", "- nodes:"]
    for n in nodes:
        lines.append("  - {name: %s, host: %s, port: %d}" % (n["name"], n["host"], n["port"]))
    lines.append("- fetch_probability: %r" % fetch_p)
    lines.append("- timeout_ms: %d" % timeout_ms)
    lines.append("- interpolation: %s" % interp)
    lines.append("- divergence_threshold: %r" % thr)
    lines.append("- constant: { value: %r }" % (extra if extra is not None else 0.5))
    lines.append("- clock: 0")
    lines.append("- loss: 0")
    with open(path, "wt") as f:
        f.write("\n".join(lines) + "\n")


def make_nodes(G, base_port=46000):
    return [{"name": "w%d" % (g + 1), "host": "localhost", "port": base_port + g} for g in range(G)]


def new_connection(cfg_path, name, seed, real_tx):
    """Builds the reference DpwaConnection through its real __init__ (dpwa.py:54-93)."""
    if real_tx:
        rdpwa.TxThread = rconn.TxThread
    else:
        rdpwa.TxThread = FakeTx
    RNG.rngs[name] = random.Random(seed)
    conn = rdpwa.DpwaConnection(name, cfg_path)
    if real_tx:
        RNG.by_thread[conn.tx.ident] = name
    return conn


class FakeTx:
    """Scripted TxThread for the policy traces: fetch_wait returns a queued reply."""

    def __init__(self, timeout_ms):
        self.replies = []
        self.peers = []

    def add_peer(self, name, host, port):
        self.peers.append(name)

    def start(self):
        pass

    def fetch_send(self):
        pass

    def fetch_wait(self):
        return self.replies.pop(0)


def jnum(x):
    """JSON-safe float/int (keeps int-ness; encodes non-finite as strings)."""
    if isinstance(x, (bool, np.bool_)):
        return bool(x)
    if isinstance(x, (int, np.integer)):
        return int(x)
    x = float(x)
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    return x


def fbits(x):
    return float(x).hex()


# ----------------------------------------------------------------------------
# A. fp32 lerp through the reference adapter
# ----------------------------------------------------------------------------
class Net(torch.nn.Module):
    def __init__(self, shapes, dtype=torch.float32):
        super().__init__()
        for i, s in enumerate(shapes):
            self.register_parameter("p%d" % i, torch.nn.Parameter(torch.zeros(s, dtype=dtype)))


class CaptureConn:
    def update_send(self, blob, loss):
        self.blob = blob


class ScriptConn:
    def __init__(self, blob, factor):
        self.blob, self.factor = blob, factor

    def update_wait(self, loss):
        return self.blob, self.factor


def adapter_for(net, conn):
    a = object.__new__(DpwaPyTorchAdapter)
    a._net = net
    a._conn = conn
    return a


def flat_params(net):
    return np.concatenate([p.detach().numpy().reshape(-1) for _, p in net.named_parameters()])


def load_flat(net, flat):
    off = 0
    for _, p in net.named_parameters():
        n = p.numel()
        p.data = torch.from_numpy(flat[off:off + n].copy()).view(p.shape)
        off += n


SPECIALS = np.array([0.0, -0.0, 1e-40, -1e-40, 1.4e-45, 3.4e38, -3.4e38, np.inf, -np.inf, np.nan,
                     1.0, -1.0, 1e-30, 65504.0, 1.0000001, 0.1], dtype=np.float32)


def gen_lerp_f32():
    shapes = [(5, 7), (5,), (4, 3, 3, 3), (4,), (1,), (1027,), (64, 64), (3, 33)]
    rng = np.random.default_rng(20261015)
    n = sum(int(np.prod(s)) for s in shapes)
    param = (rng.standard_normal(n) * 10 ** rng.uniform(-3, 3, n)).astype(np.float32)
    peer = (rng.standard_normal(n) * 10 ** rng.uniform(-3, 3, n)).astype(np.float32)
    # near-cancellation pairs, where FMA contraction would change the result
    k = 512
    peer[100:100 + k] = -param[100:100 + k] * np.float32(1.0 + 1e-6)
    param[2000:2000 + len(SPECIALS)] = SPECIALS
    peer[2000:2000 + len(SPECIALS)] = SPECIALS[::-1]
    peer[2100:2100 + len(SPECIALS)] = SPECIALS
    factors = [0.5, 1.0 / 3.0, 0.125, 0.7, 0.9999, 2.0 / 7.0, 0.0, 1.0, 0.1, 1e-9]

    peer_net = Net(shapes)
    load_flat(peer_net, peer)
    cap = CaptureConn()
    adapter_for(peer_net, cap).update_send(0.0)       # pytorch.py:42-53 -> pickled dict of bytes
    outs = []
    for f in factors:
        me = Net(shapes)
        load_flat(me, param)
        adapter_for(me, ScriptConn(cap.blob, f)).update_wait(1.0)   # pytorch.py:55-68
        outs.append(flat_params(me))
    np.savez_compressed(os.path.join(OUT, "lerp_f32.npz"), param=param, peer=peer,
                        factors=np.array(factors, dtype=np.float64), out=np.stack(outs),
                        shapes=np.array(json.dumps(shapes)))
    print("lerp_f32: %d elems x %d factors" % (n, len(factors)))


def gen_lerp_bf16():
    """torch-eager bf16: bf16(bf16(f*t) + bf16((1-f)*p)).  NOT reference output."""
    rng = np.random.default_rng(7)
    n = 8192 + 13
    p = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(torch.bfloat16)
    t = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(torch.bfloat16)
    t[:512] = -p[:512]
    factors = [0.5, 1.0 / 3.0, 0.125, 0.7, 0.9999, 2.0 / 7.0, 0.0, 1.0]
    outs = [(f * t + (1 - f) * p).view(torch.int16).numpy().view(np.uint16) for f in factors]
    np.savez_compressed(os.path.join(OUT, "lerp_bf16.npz"),
                        param=p.view(torch.int16).numpy().view(np.uint16),
                        peer=t.view(torch.int16).numpy().view(np.uint16),
                        factors=np.array(factors), out=np.stack(outs))
    print("lerp_bf16: %d elems" % n)


# ----------------------------------------------------------------------------
# C. policy traces: factor / clock / Bernoulli through DpwaConnection
# ----------------------------------------------------------------------------
def gen_policy(tmp):
    cases = []
    interps = [("constant", 0.5), ("constant", 0.3), ("constant", 1.0), ("clock", None), ("loss", None)]
    for interp, val in interps:
        for thr in (0.0, 0.5):
            for fp in (1.0, 0.7):
                for seed in (0, 1):
                    cases.append((interp, val, thr, fp, seed))
    out = []
    for ci, (interp, val, thr, fp, seed) in enumerate(cases):
        cfg = os.path.join(tmp, "policy_%d.yaml" % ci)
        write_config(cfg, make_nodes(3), fp, interp, thr, extra=val)
        conn = new_connection(cfg, "w2", seed, real_tx=False)
        RNG.set_current("w2")
        script = random.Random(1000 + ci)
        rounds = []
        peer_clock = 0
        for r in range(48):
            send_loss = script.choice([script.uniform(0.0, 2.0), script.uniform(0.0, 0.6), 0.5,
                                       float(script.randint(0, 3))])
            conn.update_send(b"blob", send_loss)
            rec = {"send_loss": jnum(send_loss), "fetching": conn.fetching,
                   "pub_clock": jnum(conn.rx.state["clock"]), "pub_loss": jnum(conn.rx.state["loss"])}
            peer_clock = script.choice([peer_clock + 1, peer_clock + script.randint(1, 5),
                                        peer_clock + 0.5 * script.random(), float(r) / 3.0 + 1])
            peer_loss = script.choice([script.uniform(0.01, 2.0), 0.25, script.uniform(0, 0.5)])
            has = script.random() >= 0.1
            wait_loss = script.choice([script.uniform(0.01, 2.0), script.uniform(0.01, 0.6), 0.5])
            if interp == "loss" and script.random() < 0.05:
                wait_loss, peer_loss = 0.0, 0.0
            if conn.fetching:
                conn.tx.replies.append(({"clock": peer_clock, "loss": peer_loss}, b"p" if has else None))
            rec.update({"peer_clock": jnum(peer_clock), "peer_loss": jnum(peer_loss), "has_payload": has,
                        "wait_loss": jnum(wait_loss)})
            try:
                payload, factor = conn.update_wait(wait_loss)
                rec.update({"averaged": payload is not None, "factor": jnum(factor),
                            "factor_hex": fbits(factor), "clock_after": jnum(conn.clock),
                            "clock_hex": fbits(conn.clock), "raises": None})
            except ZeroDivisionError:
                rec.update({"averaged": False, "factor": None, "clock_after": jnum(conn.clock),
                            "clock_hex": fbits(conn.clock), "raises": "ZeroDivisionError"})
                conn.fetching = False
            rounds.append(rec)
        out.append({"interpolation": interp, "value": val, "divergence_threshold": thr,
                    "fetch_probability": fp, "seed": seed, "rounds": rounds})
    with open(os.path.join(OUT, "policy.json"), "wt") as f:
        json.dump({"source": "reference dpwa/dpwa.py:101-156 + dpwa/interpolation.py via DpwaConnection",
                   "cases": out}, f, indent=0)
    print("policy: %d cases" % len(out))


# ----------------------------------------------------------------------------
# D. peer selection + flow control under scripted faults (real TxThread)
# ----------------------------------------------------------------------------
PROFILES = {
    # (P(connect ok), P(refused), P(error)) , (payload, empty, timeout, error)
    "clean": ((1.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0)),
    "startup": ((0.7, 0.3, 0.0), (0.6, 0.4, 0.0, 0.0)),
    "flaky": ((0.8, 0.18, 0.02), (0.55, 0.15, 0.28, 0.02)),
    "dying": ((0.7, 0.15, 0.15), (0.5, 0.1, 0.2, 0.2)),
}


def pick(rng, names, weights):
    u = rng.random()
    acc = 0.0
    for n, w in zip(names, weights):
        acc += w
        if u < acc:
            return n
    return names[-1]


def gen_peer_select(tmp):
    out = []
    ci = 0
    for G in (2, 4, 8):
        for fp in (1.0, 0.7):
            for prof in PROFILES:
                for seed in (3, 11):
                    ci += 1
                    nodes = make_nodes(G, base_port=47000 + 16 * ci)
                    for n in nodes:
                        ADDR2NAME[(n["host"], n["port"])] = n["name"]
                    cfg = os.path.join(tmp, "sel_%d.yaml" % ci)
                    write_config(cfg, nodes, fp, "clock", 0.0)
                    me = "w%d" % (1 + (seed % G))
                    conn = new_connection(cfg, me, seed, real_tx=True)
                    peers = [n["name"] for n in nodes if n["name"] != me]
                    env_rng = random.Random(seed * 7919 + G)
                    (pc, pr, pe), (qp, qe, qt, qx) = PROFILES[prof]
                    ENV.gate = None
                    ENV.connect_fn = lambda peer: pick(env_rng, ["ok", "refused", "error"], [pc, pr, pe])
                    ENV.request_fn = lambda peer: pick(env_rng, ["payload", "empty", "timeout", "error"],
                                                       [qp, qe, qt, qx])
                    ENV.reply_fn = lambda peer: ({"clock": 1 + int(peer[1:]), "loss": 0.5}, b"payload")
                    rounds = []
                    for r in range(40):
                        RNG.set_current(me)
                        ENV.logs[me] = []
                        conn.update_send(b"mine", 1.0)
                        fetching = conn.fetching
                        payload, factor = conn.update_wait(1.0)
                        scores = []
                        for p in peers:
                            w = conn.tx.peers.get(p)
                            scores.append(None if w is None else w.flow_control_score)
                        rounds.append({"fetching": fetching, "attempts": list(ENV.logs[me]),
                                       "data": payload is not None, "factor_hex": fbits(factor),
                                       "clock_hex": fbits(conn.clock), "scores": scores})
                    conn.tx._queue.put(False)
                    out.append({"G": G, "me": me, "peers": peers, "fetch_probability": fp,
                                "profile": prof, "seed": seed, "rounds": rounds})
    with open(os.path.join(OUT, "peer_select.json"), "wt") as f:
        json.dump({"source": "reference dpwa/conn.py:224-317 TxThread + dpwa/dpwa.py:101-156",
                   "cases": out}, f, indent=0)
    print("peer_select: %d cases" % len(out))


def gen_peer_add(tmp):
    """TxThread with peers removed by errors and put back by DpwaConnection.add_peer
    (dpwa.py:95-96 -> conn.py:208-213): a re-added peer is a fresh WorkerConn (score 1000,
    not connected) and a removed one re-enters the dict -- and so the per-pick randint
    order -- at the end."""
    out = []
    ci = 0
    for G in (3, 5):
        for prof in ("dying", "flaky"):
            for seed in (3, 11):
                ci += 1
                nodes = make_nodes(G, base_port=48000 + 16 * ci)
                for n in nodes:
                    ADDR2NAME[(n["host"], n["port"])] = n["name"]
                cfg = os.path.join(tmp, "add_%d.yaml" % ci)
                write_config(cfg, nodes, 1.0, "clock", 0.0)
                me = "w%d" % (1 + (seed % G))
                conn = new_connection(cfg, me, seed, real_tx=True)
                peers = [n["name"] for n in nodes if n["name"] != me]
                env_rng = random.Random(seed * 104729 + G)
                (pc, pr, pe), (qp, qe, qt, qx) = PROFILES[prof]
                ENV.gate = None
                ENV.connect_fn = lambda peer: pick(env_rng, ["ok", "refused", "error"], [pc, pr, pe])
                ENV.request_fn = lambda peer: pick(env_rng, ["payload", "empty", "timeout", "error"],
                                                   [qp, qe, qt, qx])
                ENV.reply_fn = lambda peer: ({"clock": 1 + int(peer[1:]), "loss": 0.5}, b"payload")
                rounds = []
                for r in range(40):
                    adds = []
                    if r in (8, 16, 24, 32):        # put every removed peer back
                        adds = [p for p in peers if p not in conn.tx.peers]
                    if r in (12, 28):               # re-add a live peer: its record is reset
                        live = [p for p in peers if p in conn.tx.peers]
                        adds += live[-1:]
                    for p in adds:
                        node = [n for n in nodes if n["name"] == p][0]
                        conn.add_peer(p, node["host"], node["port"])
                    RNG.set_current(me)
                    ENV.logs[me] = []
                    conn.update_send(b"mine", 1.0)
                    fetching = conn.fetching
                    payload, factor = conn.update_wait(1.0)
                    scores = []
                    for p in peers:
                        w = conn.tx.peers.get(p)
                        scores.append(None if w is None else w.flow_control_score)
                    rounds.append({"add_peer": adds, "fetching": fetching, "attempts": list(ENV.logs[me]),
                                   "data": payload is not None, "scores": scores,
                                   "order": list(conn.tx.peers.keys())})
                conn.tx._queue.put(False)
                out.append({"G": G, "me": me, "peers": peers, "fetch_probability": 1.0,
                            "profile": prof, "seed": seed, "rounds": rounds})
    with open(os.path.join(OUT, "peer_add.json"), "wt") as f:
        json.dump({"source": "reference dpwa/dpwa.py:95-99 add_peer/remove_peer + dpwa/conn.py:208-317 TxThread",
                   "cases": out}, f, indent=0)
    print("peer_add: %d cases" % len(out))


# ----------------------------------------------------------------------------
# E. lock-step G-learner gossip with data through the real adapter
# ----------------------------------------------------------------------------
GOSSIP_SHAPES = [(8, 5), (8,), (4, 2, 3, 3), (4,), (4,), (3, 17), (3,)]


GOSSIP_CASES = [("constant", 0.5, 0.0, 1.0, 4), ("clock", None, 0.0, 1.0, 4),
                ("loss", None, 0.5, 0.7, 4), ("constant", 0.25, 0.5, 0.7, 3), ("clock", None, 0.5, 1.0, 8)]
# the loop order resident parameters need (update_send -> update_wait -> step): G = 3 and 4,
# clock and loss interpolation, fetch_probability 0.7
GOSSIP_STEP_AFTER_WAIT_CASES = [("clock", None, 0.0, 0.7, 3), ("loss", None, 0.5, 0.7, 4),
                                ("clock", None, 0.5, 0.7, 4), ("loss", None, 0.0, 0.7, 3)]


def gen_gossip(tmp, step_after_wait=False):
    """Lock-step rounds through the real adapter.  README order (README.md:18-29,
    main.py:130-145): update_send, training step, update_wait.  step_after_wait: the same
    adapter calls with the step after update_wait (update_send, update_wait, step -- the
    reference runs either order: pytorch.py:42-68 and dpwa.py:104-156 never look at what
    happened in between); the recorded parameters are then the ones update_wait left, before
    the round's step."""
    npz = {}
    meta = {"shapes": GOSSIP_SHAPES, "cases": [],
            "order": "update_send, update_wait, step" if step_after_wait else "update_send, step, update_wait"}
    cases = GOSSIP_STEP_AFTER_WAIT_CASES if step_after_wait else GOSSIP_CASES
    base_port = 50000 if step_after_wait else 49000
    seed_base = 300 if step_after_wait else 100
    n = sum(int(np.prod(s)) for s in GOSSIP_SHAPES)
    T = 8
    for ci, (interp, val, thr, fp, G) in enumerate(cases):
        nodes = make_nodes(G, base_port=base_port + 32 * ci)
        for nd in nodes:
            ADDR2NAME[(nd["host"], nd["port"])] = nd["name"]
        cfg = os.path.join(tmp, "gossip_%d.yaml" % ci)
        write_config(cfg, nodes, fp, interp, thr, extra=val)
        rng = np.random.default_rng(seed_base + ci)
        names = [nd["name"] for nd in nodes]
        init = rng.standard_normal((G, n)).astype(np.float32)
        deltas = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
        lrng = random.Random(seed_base - 45 + ci)
        send_loss = [[2 * math.exp(-r / 3.0) + 0.05 * lrng.random() for _ in range(G)] for r in range(T)]
        wait_loss = [[2 * math.exp(-(r + 0.5) / 3.0) + 0.05 * lrng.random() for _ in range(G)] for r in range(T)]
        nets, adapters, conns = [], [], []
        addr = {nd["name"]: (nd["host"], nd["port"]) for nd in nodes}
        for g, name in enumerate(names):
            net = Net(GOSSIP_SHAPES)
            load_flat(net, init[g])
            conn = new_connection(cfg, name, 10 * seed_base + g, real_tx=True)
            nets.append(net)
            conns.append(conn)
            adapters.append(adapter_for(net, conn))

        def reply(peer):
            rx = FakeRx.registry[addr[peer]]
            with rx.lock:
                return copy.deepcopy(rx.state), rx.payload

        ENV.connect_fn = lambda peer: "ok"
        ENV.request_fn = lambda peer: "payload"
        ENV.reply_fn = reply
        params = np.zeros((T, G, n), np.float32)
        clocks = np.zeros((T, G), np.float64)
        factors = np.zeros((T, G), np.float64)
        fetching = np.zeros((T, G), np.bool_)
        picks = [[None] * G for _ in range(T)]
        for r in range(T):
            ENV.gate = threading.Event()
            for g in range(G):
                RNG.set_current(names[g])
                ENV.logs[names[g]] = []
                adapters[g].update_send(send_loss[r][g])          # publish + Bernoulli + fetch_send
                fetching[r, g] = conns[g].fetching
            ENV.gate.set()                                       # every learner has published round r

            def train():
                for g in range(G):
                    with torch.no_grad():                        # the "training step"
                        off = 0
                        for _, p in nets[g].named_parameters():
                            k = p.numel()
                            p.data.add_(torch.from_numpy(deltas[r, g, off:off + k]).view(p.shape))
                            off += k
            if not step_after_wait:
                train()
            for g in range(G):
                RNG.set_current(names[g])
                c = conns[g]
                # capture factor by wrapping this connection's update_wait
                holder = {}
                orig = c.update_wait

                def wrapped(loss, orig=orig, holder=holder):
                    res = orig(loss)
                    holder["factor"] = res[1]
                    return res

                c.update_wait = wrapped
                adapters[g].update_wait(wait_loss[r][g])
                del c.update_wait
                factors[r, g] = holder["factor"]
                clocks[r, g] = c.clock
                params[r, g] = flat_params(nets[g])
            for g in range(G):
                picks[r][g] = [a["peer"] for a in ENV.logs[names[g]]]
            if step_after_wait:
                train()
        for c in conns:
            c.tx._queue.put(False)
        ENV.gate = None
        key = "c%d" % ci
        npz[key + "_init"] = init
        npz[key + "_deltas"] = deltas
        npz[key + "_params"] = params
        npz[key + "_clocks"] = clocks
        npz[key + "_factors"] = factors
        npz[key + "_fetching"] = fetching
        meta["cases"].append({"key": key, "interpolation": interp, "value": val,
                              "divergence_threshold": thr, "fetch_probability": fp, "G": G,
                              "names": names, "seeds": [10 * seed_base + g for g in range(G)],
                              "send_loss": send_loss, "wait_loss": wait_loss, "picks": picks})
    stem = "gossip_step_after_wait" if step_after_wait else "gossip"
    np.savez_compressed(os.path.join(OUT, stem + ".npz"), **npz)
    with open(os.path.join(OUT, stem + ".json"), "wt") as f:
        json.dump(meta, f, indent=0)
    print("%s: %d cases" % (stem, len(meta["cases"])))


def gen_gossip_step_after_wait(tmp):
    gen_gossip(tmp, step_after_wait=True)


# configs[1]'s self-peer: one learner whose YAML lists a second node entry at its own host:port,
# so its TxThread dials its own RxThread (conn.py:246-251 -> 98-110) and averages with the
# snapshot it published.  (interpolation, constant value, divergence threshold, fetch_probability)
GOSSIP_SELF_CASES = [("constant", 0.5, 0.0, 1.0), ("clock", None, 0.5, 0.7), ("loss", None, 0.5, 1.0),
                     ("constant", 0.25, 0.0, 0.7)]


def gen_gossip_self(tmp):
    """One learner, README order (update_send, step, update_wait), nodes [w1 @ P, w1-self @ P]:
    every fetch reaches w1's own RxThread.  The fake socket layer routes a connection by address,
    as TCP does (FakeRx.registry), so the reference alone decides picks, factors and clocks."""
    npz = {}
    meta = {"shapes": GOSSIP_SHAPES, "cases": [], "order": "update_send, step, update_wait",
            "nodes": "w1 and w1-self at one host:port (the learner's own RxThread)"}
    n = sum(int(np.prod(s_)) for s_ in GOSSIP_SHAPES)
    T = 10
    for ci, (interp, val, thr, fp) in enumerate(GOSSIP_SELF_CASES):
        port = 51000 + ci
        nodes = [{"name": "w1", "host": "localhost", "port": port},
                 {"name": "w1-self", "host": "localhost", "port": port}]
        ADDR2NAME[("localhost", port)] = "w1-self"      # only w1 dials, and only w1-self is its peer
        cfg = os.path.join(tmp, "gossip_self_%d.yaml" % ci)
        write_config(cfg, nodes, fp, interp, thr, extra=val)
        rng = np.random.default_rng(500 + ci)
        init = rng.standard_normal((1, n)).astype(np.float32)
        deltas = (0.01 * rng.standard_normal((T, 1, n))).astype(np.float32)
        lrng = random.Random(455 + ci)
        send_loss = [[2 * math.exp(-r / 3.0) + 0.05 * lrng.random()] for r in range(T)]
        wait_loss = [[2 * math.exp(-(r + 0.5) / 3.0) + 0.05 * lrng.random()] for r in range(T)]
        net = Net(GOSSIP_SHAPES)
        load_flat(net, init[0])
        seed = 5000 + ci
        conn = new_connection(cfg, "w1", seed, real_tx=True)
        adapter = adapter_for(net, conn)

        def reply(peer):
            rx = FakeRx.registry[("localhost", port)]
            with rx.lock:
                return copy.deepcopy(rx.state), rx.payload

        ENV.connect_fn = lambda peer: "ok"
        ENV.request_fn = lambda peer: "payload"
        ENV.reply_fn = reply
        ENV.gate = None
        params = np.zeros((T, 1, n), np.float32)
        clocks = np.zeros((T, 1), np.float64)
        factors = np.zeros((T, 1), np.float64)
        fetching = np.zeros((T, 1), np.bool_)
        picks = [[None] for _ in range(T)]
        for r in range(T):
            RNG.set_current("w1")
            ENV.logs["w1"] = []
            adapter.update_send(send_loss[r][0])
            fetching[r, 0] = conn.fetching
            with torch.no_grad():                        # the "training step"
                off = 0
                for _, p_ in net.named_parameters():
                    k = p_.numel()
                    p_.data.add_(torch.from_numpy(deltas[r, 0, off:off + k]).view(p_.shape))
                    off += k
            holder = {}
            orig = conn.update_wait

            def wrapped(loss, orig=orig, holder=holder):
                res = orig(loss)
                holder["factor"] = res[1]
                return res

            conn.update_wait = wrapped
            adapter.update_wait(wait_loss[r][0])
            del conn.update_wait
            factors[r, 0] = holder["factor"]
            clocks[r, 0] = conn.clock
            params[r, 0] = flat_params(net)
            picks[r][0] = [a["peer"] for a in ENV.logs["w1"]]
        conn.tx._queue.put(False)
        key = "c%d" % ci
        npz[key + "_init"] = init
        npz[key + "_deltas"] = deltas
        npz[key + "_params"] = params
        npz[key + "_clocks"] = clocks
        npz[key + "_factors"] = factors
        npz[key + "_fetching"] = fetching
        meta["cases"].append({"key": key, "interpolation": interp, "value": val, "divergence_threshold": thr,
                              "fetch_probability": fp, "G": 1, "names": ["w1"], "nodes": ["w1", "w1-self"],
                              "serves": {"w1-self": 0}, "seeds": [seed], "send_loss": send_loss,
                              "wait_loss": wait_loss, "picks": picks})
    np.savez_compressed(os.path.join(OUT, "gossip_self.npz"), **npz)
    with open(os.path.join(OUT, "gossip_self.json"), "wt") as f:
        json.dump(meta, f, indent=0)
    print("gossip_self: %d cases" % len(meta["cases"]))


# ----------------------------------------------------------------------------
# F. wire frames
# ----------------------------------------------------------------------------
def gen_wire():
    samples = []
    for (mtype, msg, payload) in [(1, None, None), (1, {"clock": 3, "loss": 0.25}, bytes(range(40))),
                                  (1, {"clock": 7.5, "loss": 1e-3}, b""), (2, None, b"\x00" * 17)]:
        a, b = socket.socketpair()
        rmsg.send_message(a, mtype, msg, payload)
        a.shutdown(socket.SHUT_WR)
        raw = b""
        while True:
            chunk = b.recv(1 << 16)
            if not chunk:
                break
            raw += chunk
        a.close()
        b.close()
        a, b = socket.socketpair()
        a.sendall(raw)
        t, m, p = rmsg.recv_message(b)
        a.close()
        b.close()
        samples.append({"type": mtype, "message": msg, "payload_hex": None if payload is None else payload.hex(),
                        "frame_hex": raw.hex(), "decoded": {"type": t, "message": m,
                                                            "payload_hex": None if p is None else p.hex()}})
    with open(os.path.join(OUT, "wire.json"), "wt") as f:
        json.dump({"source": "reference dpwa/messaging.py:24-94", "header_fmt": rmsg.HEADER_FMT,
                   "header_len": rmsg.HEADER_LEN, "chunk_size": rmsg.CHUNK_SIZE, "samples": samples}, f,
                  indent=0)
    print("wire: %d samples" % len(samples))


def gen_wire_adapter():
    """RxThread replies carrying a real adapter blob: header + pickle(state) +
    pickle({name: raw fp32 bytes}) (pytorch.py:42-53 -> dpwa.py:115-116 -> conn.py:110)."""
    shapes = [(4, 3), (5,), (2, 2, 2)]
    rng = np.random.default_rng(77)
    n = sum(int(np.prod(s_)) for s_ in shapes)
    flat = rng.standard_normal(n).astype(np.float32)
    net = Net(shapes)
    load_flat(net, flat)
    cap = CaptureConn()
    adapter_for(net, cap).update_send(0.0)
    frames = []
    for state in ({"clock": 3, "loss": 0.5}, {"clock": 7.25, "loss": 1e-3}):
        a, b = socket.socketpair()
        rmsg.send_message(a, rconn.MESSAGE_TYPE_FETCH_PARAMETERS, state, cap.blob)
        a.shutdown(socket.SHUT_WR)
        raw = b""
        while True:
            chunk = b.recv(1 << 16)
            if not chunk:
                break
            raw += chunk
        a.close()
        b.close()
        frames.append({"state": state, "frame_hex": raw.hex()})
    names = [nm for nm, _ in net.named_parameters()]
    with open(os.path.join(OUT, "wire_adapter.json"), "wt") as f:
        json.dump({"source": "reference adapter blob (pytorch.py:49-53) in an RxThread reply (conn.py:110)",
                   "shapes": shapes, "names": names, "flat_f32_hex": flat.tobytes().hex(),
                   "blob_hex": cap.blob.hex(), "frames": frames}, f, indent=0)
    print("wire_adapter: %d frames" % len(frames))


# ----------------------------------------------------------------------------
# G. configuration parsing
# ----------------------------------------------------------------------------
CONFIGS = {
    "four_nodes.yaml": "---\n- nodes:\n  - {name: w1, host: localhost, port: 45000}\n"
                       "  - {name: w2, host: localhost, port: 45001}\n"
                       "  - {name: w3, host: localhost, port: 45002}\n"
                       "  - {name: w4, host: localhost, port: 45003}\n"
                       "- fetch_probability: 1\n- timeout_ms: 2500\n- interpolation: constant\n"
                       "- divergence_threshold: 0.2\n- constant: { value: 0.5 }\n- clock: 0\n- loss: 0\n",
    "clock_eight.yaml": "---\n- nodes:\n" + "".join(
        "  - {name: gpu%d, host: 127.0.0.1, port: %d}\n" % (i, 45100 + i) for i in range(8)) +
        "- fetch_probability: 0.7\n- timeout_ms: 100\n- interpolation: clock\n"
        "- divergence_threshold: 0\n- constant: { value: 0.25 }\n- clock: 0\n- loss: 0\n",
    "loss_two.yaml": "- nodes:\n  - {name: a, host: localhost, port: 45200}\n"
                     "  - {name: b, host: localhost, port: 45201}\n"
                     "- interpolation: loss\n- loss: 0\n- timeout_ms: 2500\n"
                     "- fetch_probability: 0.5\n- divergence_threshold: 0.5\n",
}


def _generated_configs():
    """Node lists written by dpwa_amd.launch (this repository's launcher, with the per-node
    gpu: key): the reference must load them (tests/test_config.py)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from dpwa_amd.launch import config_text
    return {"launch_gpu.yaml": config_text(["w0", "w1", "w2"], gpus=[0, 1, 2], interpolation="clock",
                                           divergence_threshold=0.5),
            "launch_plain.yaml": config_text(["w1", "w2"], fetch_probability=0.7, interpolation="loss")}


def gen_config(tmp):
    out = {}
    for fname, text in list(CONFIGS.items()) + list(_generated_configs().items()):
        path = os.path.join(tmp, fname)
        with open(path, "wt") as f:
            f.write(text)
        c = rdpwa.DpwaConfiguration(path)
        rec = {"text": text, "config": c.config, "nodes": c.get_nodes(),
               "interpolation": list(c.get_interpolation()), "timeout_ms": c.get_timeoutms(),
               "fetch_probability": c.get_fetch_probability(),
               "divergence_threshold": c.get_divergence_threshold(), "connections": {}}
        for node in c.get_nodes():
            conn = new_connection(path, node["name"], 0, real_tx=False)
            rec["connections"][node["name"]] = {
                "me": conn.me.__dict__, "peers": [p.__dict__ for p in conn.peers],
                "tx_peers": conn.tx.peers, "interp_class": type(conn.interpolation).__name__,
                "divergence_threshold": conn.divergence_threshold, "clock": conn.clock}
        out[fname] = rec
    # error behaviour: constant value out of range raises AssertionError (interpolation.py:10)
    bad = os.path.join(tmp, "bad.yaml")
    with open(bad, "wt") as f:
        f.write(CONFIGS["four_nodes.yaml"].replace("value: 0.5", "value: 1.5"))
    try:
        new_connection(bad, "w1", 0, real_tx=False)
        err = None
    except AssertionError:
        err = "AssertionError"
    out["_bad_constant"] = {"text": open(bad).read(), "raises": err}
    bad2 = os.path.join(tmp, "bad2.yaml")
    with open(bad2, "wt") as f:
        f.write(CONFIGS["four_nodes.yaml"].replace("interpolation: constant", "interpolation: cubic")
                + "- cubic: 0\n")
    try:
        new_connection(bad2, "w1", 0, real_tx=False)
        err = None
    except KeyError:
        err = "KeyError"
    out["_bad_method"] = {"text": open(bad2).read(), "raises": err}
    with open(os.path.join(OUT, "config.json"), "wt") as f:
        json.dump({"source": "reference dpwa/dpwa.py:29-93", "files": out}, f, indent=0)
    print("config: %d files" % len(out))


def main():
    only = sys.argv[1:]
    if only:     # regenerate just the named fixtures, e.g. `make_golden.py peer_add`
        with tempfile.TemporaryDirectory() as tmp:
            for name in only:
                fn = globals()["gen_" + name]
                fn(tmp) if fn.__code__.co_argcount else fn()
        os._exit(0)
    with tempfile.TemporaryDirectory() as tmp:
        gen_lerp_f32()
        gen_lerp_bf16()
        gen_policy(tmp)
        gen_peer_select(tmp)
        gen_peer_add(tmp)
        gen_gossip(tmp)
        gen_gossip_step_after_wait(tmp)
        gen_gossip_self(tmp)
        gen_wire()
        gen_wire_adapter()
        gen_config(tmp)
    os._exit(0)   # reference TxThreads are non-daemon and never exit on their own (conn.py:170-172)


if __name__ == "__main__":
    sys.stdout.flush()
    main()
