"""Wire bridge on the GPU: a GPU learner serves its HBM snapshot in the
reference's frame format and averages with snapshots that arrive over TCP."""
import socket
import threading
import time

import numpy as np
import pytest
import torch

from dpwa_amd import DpwaPyTorchAdapter, wire
from dpwa_amd.bridge import SnapshotCodec, WireConnection
from oracle import gossip as ogossip
from oracle import lerp as olerp
from tests.helpers import load_json
from tests.test_gpu_gossip import Net

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def wire_cfg(path, names, ports, fp=1.0, interp="constant", value=0.5):
    lines = ["- nodes:"] + ["  - {name: %s, host: 127.0.0.1, port: %d}" % (n, p) for n, p in zip(names, ports)]
    lines += ["- fetch_probability: %r" % fp, "- timeout_ms: 5000", "- interpolation: %s" % interp,
              "- divergence_threshold: 0", "- constant: { value: %r }" % value, "- clock: 0", "- loss: 0"]
    path.write_text("\n".join(lines) + "\n")


def recv_all(sock, n):
    out = b""
    while len(out) < n:
        chunk = sock.recv(n - len(out))
        assert chunk
        out += chunk
    return out


def fixture_net():
    fx = load_json("wire_adapter.json")
    net = Net([tuple(s) for s in fx["shapes"]]).to(DEV)
    flat = np.frombuffer(bytes.fromhex(fx["flat_f32_hex"]), dtype=np.float32)
    off = 0
    with torch.no_grad():
        for _, p in net.named_parameters():
            p.copy_(torch.from_numpy(flat[off:off + p.numel()].copy()).view(p.shape))
            off += p.numel()
    return fx, net, flat


def test_served_frames_match_reference_rxthread(tmp_path):
    fx, net, _ = fixture_net()
    ports = [free_port(), free_port()]
    cfg = tmp_path / "serve.yaml"
    wire_cfg(cfg, ["g", "other"], ports, fp=0.0)
    ad = DpwaPyTorchAdapter(net, "g", str(cfg), transport="wire", seed=1)
    for fr in fx["frames"]:
        st = fr["state"]
        ad.connection._learner.write_clock(float(st["clock"]) - 1) if ad.connection._learner else None
        if ad.connection._learner is None:           # bind on the first publish, then set the clock
            ad.update_send(st["loss"])
            ad.connection._learner.write_clock(float(st["clock"]) - 1)
        ad.update_send(st["loss"])                   # clock += 1 -> st["clock"]
        c = socket.create_connection(("127.0.0.1", ports[0]))
        c.sendall(wire.encode(1))
        want = bytes.fromhex(fr["frame_hex"])
        assert recv_all(c, len(want)) == want
        c.close()
    ad.connection.close()


def test_fetch_from_reference_format_peer(tmp_path):
    """A 'reference node' that answers with the reference's own reply bytes: the GPU learner
    parses the blob, stages it in HBM and averages bit-exactly like the reference adapter."""
    fx, net, flat = fixture_net()
    frame = bytes.fromhex(fx["frames"][1]["frame_hex"])          # clock 7.25, loss 1e-3
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(4)

    def serve():
        c, _ = srv.accept()
        while True:
            hdr = c.recv(wire.HEADER_LEN)
            if not hdr:
                break
            c.sendall(frame)
        c.close()

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    ports = [free_port(), srv.getsockname()[1]]
    cfg = tmp_path / "fetch.yaml"
    wire_cfg(cfg, ["g", "ref"], ports, interp="clock")
    mine = (np.arange(flat.size, dtype=np.float32) - 7) / 3
    off = 0
    with torch.no_grad():
        for _, p in net.named_parameters():
            p.copy_(torch.from_numpy(mine[off:off + p.numel()]).view(p.shape))
            off += p.numel()
    ad = DpwaPyTorchAdapter(net, "g", str(cfg), transport="wire", seed=3)
    ad.update_send(1.0)                                          # clock 1
    ad.update_wait(1.0)
    f = 7.25 / (1.0 + 7.25)                                      # clock interpolation
    want = olerp.lerp_f32(mine, flat, f)
    got = torch.cat([p.detach().reshape(-1) for _, p in net.named_parameters()]).cpu().numpy()
    assert olerp.bits_equal(got, want)
    assert ad.connection.clock == f * 7.25 + (1 - f) * 1.0
    ad.connection.close()
    srv.close()


def test_two_gpu_learners_gossip_over_tcp(tmp_path):
    rng = np.random.default_rng(8)
    G, n, T = 3, 20_000, 6
    names = ["t%d" % g for g in range(G)]
    ports = [free_port() for _ in range(G)]
    cfg = tmp_path / "tcp.yaml"
    wire_cfg(cfg, names, ports, fp=0.8, interp="clock")
    init = rng.standard_normal((G, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    send = [[1.0] * G for _ in range(T)]
    wait = [[1.0] * G for _ in range(T)]
    seeds = [70 + g for g in range(G)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, 0.8, seeds)
    conns = [WireConnection(names[g], str(cfg), codec=SnapshotCodec.single("w", n), seed=seeds[g], eager=False)
             for g in range(G)]
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    for r in range(T):
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g])
        torch.cuda.synchronize()
        for g in range(G):
            flats[g].add_(torch.from_numpy(deltas[r, g]).to(DEV))
        for g in range(G):
            conns[g].update_wait_average(flats[g], wait[r][g])
        torch.cuda.synchronize()
    for g in range(G):
        assert olerp.bits_equal(flats[g].cpu().numpy(), exp["params"][-1, g]), g
        assert conns[g].clock == exp["clocks"][-1, g]
        conns[g].close()


def test_served_snapshots_are_never_torn_while_publishing(tmp_path):
    """Replies are sent from page-locked copies shared by concurrent readers: while the learner
    keeps publishing, every reply three clients receive is one whole published snapshot (each
    publish is a constant vector), never a mix of two."""
    n, V = 300_000, 25                       # 1.2 MB per snapshot: served as views of the copy
    ports = [free_port(), free_port()]
    cfg = tmp_path / "torn.yaml"
    wire_cfg(cfg, ["s", "absent"], ports, fp=0.0)
    conn = WireConnection("s", str(cfg), codec=SnapshotCodec.single("w", n), seed=1)
    flat = torch.zeros(n, device=DEV)
    flat.fill_(1.0)
    conn.update_send(flat, 1.0)
    torch.cuda.synchronize()
    stop = threading.Event()
    seen, errors = [], []

    def client():
        try:
            c = socket.create_connection(("127.0.0.1", ports[0]))
            while not stop.is_set():
                wire.send_frame(c, wire.MESSAGE_TYPE_FETCH_PARAMETERS)
                _, state, payload = wire.recv_frame(c)
                a = np.frombuffer(wire.param_views(payload)["w"], dtype=np.float32)
                seen.append((float(state["loss"]), float(a[0]), bool((a == a[0]).all())))
            c.close()
        except Exception as e:      # noqa: BLE001 -- reported below
            errors.append(e)

    ths = [threading.Thread(target=client) for _ in range(3)]
    for t in ths:
        t.start()
    for v in range(2, V + 1):
        flat.fill_(float(v))
        conn.update_send(flat, float(v))    # loss == value: a reply's state names its payload
        torch.cuda.synchronize()
        time.sleep(0.02)
    stop.set()
    for t in ths:
        t.join(60)
    conn.close()
    assert not errors, errors
    assert len(seen) >= V
    assert all(whole for _, _, whole in seen)
    assert all(loss == val for loss, val, _ in seen)
    assert len({val for _, val, _ in seen}) > 2           # the replies followed the publishes
