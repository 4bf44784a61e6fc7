"""Wire bridge host logic (CPU): the reference blob/frame bytes (tests/golden/wire_adapter.json,
produced by the reference adapter + messaging), the RxThread-role server, and TxThread's
fetch loop over real localhost sockets driven by the native scheduler."""
import socket

import numpy as np

from dpwa_amd import wire
from dpwa_amd.bridge import SnapshotCodec, WireServer, _Peer, fetch_loop
from dpwa_amd.sched import Scheduler
from oracle.policy import OracleLearner
from tests.helpers import load_json


def fixture_codec():
    fx = load_json("wire_adapter.json")
    numels = [int(np.prod(s)) for s in fx["shapes"]]
    offsets = list(np.cumsum([0] + numels[:-1]))
    return fx, SnapshotCodec(fx["names"], offsets, numels, sum(numels))


def test_codec_matches_reference_blob():
    fx, codec = fixture_codec()
    flat = bytes.fromhex(fx["flat_f32_hex"])
    assert codec.to_blob(flat).hex() == fx["blob_hex"]
    assert codec.from_blob(bytes.fromhex(fx["blob_hex"])) == flat


def test_codec_parts_and_views_match_the_reference_blob():
    """The zero-copy forms: to_parts concatenates to the reference's blob (also with parameters
    above pickle's 64 KiB frame target, served as views), and param_views + assemble restore the
    flat layout from it."""
    from dpwa_amd import wire
    fx, codec = fixture_codec()
    flat = bytes.fromhex(fx["flat_f32_hex"])
    assert b"".join(bytes(p) for p in codec.to_parts(bytearray(flat))).hex() == fx["blob_hex"]
    out = np.zeros(codec.total, np.float32)
    codec.assemble(wire.param_views(bytes.fromhex(fx["blob_hex"])), out)
    assert out.tobytes() == flat
    rng = np.random.default_rng(2)
    numels = [5, 40_000, 3, 70_001]                    # two of them served as views
    offsets = [0, 64, 40_064, 40_128]                  # with gaps, as the flat buffer aligns
    big = SnapshotCodec(["a", "b", "c", "d"], offsets, numels, 110_144)
    buf = rng.standard_normal(big.total).astype(np.float32)
    parts = big.to_parts(buf)
    assert sum(isinstance(p, memoryview) for p in parts) == 2
    blob = b"".join(bytes(p) for p in parts)
    assert blob == big.to_blob(buf.tobytes())
    back = np.zeros(big.total, np.float32)
    big.assemble(wire.param_views(blob), back)
    for off, n in zip(offsets, numels):
        assert np.array_equal(back[off:off + n], buf[off:off + n])


def recv_all(sock, n):
    out = b""
    while len(out) < n:
        chunk = sock.recv(n - len(out))
        assert chunk
        out += chunk
    return out


def test_server_reply_is_byte_identical_to_reference_rxthread():
    fx, codec = fixture_codec()
    blob = bytes.fromhex(fx["blob_hex"])
    for fr in fx["frames"]:
        srv = WireServer("127.0.0.1", 0, lambda st=fr["state"]: (st, blob), 2000)
        c = socket.create_connection(("127.0.0.1", srv.port))
        c.sendall(wire.encode(1))
        want = bytes.fromhex(fr["frame_hex"])
        assert recv_all(c, len(want)) == want
        c.close()
        srv.shutdown()


def test_server_empty_reply_before_publish():
    srv = WireServer("127.0.0.1", 0, lambda: None, 2000)
    c = socket.create_connection(("127.0.0.1", srv.port))
    c.sendall(wire.encode(1))
    assert recv_all(c, wire.HEADER_LEN) == wire.encode(1)
    c.close()
    srv.shutdown()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_fetch_loop_outcomes_and_flow_control_match_oracle():
    """p0 refuses (nobody listens), p1 answers without state, p2 delivers: the native
    scheduler's choices and scores follow the reference TxThread (oracle) round by round."""
    dead_port = free_port()
    empty = WireServer("127.0.0.1", 0, lambda: None, 2000)
    full = WireServer("127.0.0.1", 0, lambda: ({"clock": 1, "loss": 0.5}, b"blob"), 2000)
    peers = [_Peer("127.0.0.1", dead_port), _Peer("127.0.0.1", empty.port), _Peer("127.0.0.1", full.port)]
    names = ["p0", "p1", "p2"]
    sched = Scheduler(3, 42, 1.0)
    oracle = OracleLearner("me", names, 1.0, "clock", None, 0.0, 42)
    for r in range(25):
        assert sched.bernoulli() == (oracle.update_send(1.0) is not None and oracle.fetching)
        res = fetch_loop(sched, peers, 2000)
        st, pl, att = oracle.fetch(lambda p: "refused" if p == "p0" else "ok",
                                   lambda p: ("empty", None, None) if p == "p1" else
                                   ("payload", {"clock": 1, "loss": 0.5}, b"blob"))
        assert (res is None) == (pl is None), r
        if res is not None:
            assert names[res[0]] == att[-1]["peer"] and res[2] == b"blob" and res[1] == st
        assert sched.scores() == oracle.scores(names), r
    empty.shutdown()
    full.shutdown()
    for p in peers:
        if p.sock is not None:
            p.sock.close()


def test_fetch_loop_timeout_reconnects():
    """A peer that accepts but never answers times out: score -100, reconnect, pick again
    (conn.py:304-309)."""
    hang = socket.socket()
    hang.bind(("127.0.0.1", 0))
    hang.listen(8)
    full = WireServer("127.0.0.1", 0, lambda: ({"clock": 2, "loss": 1.0}, b"x"), 2000)
    peers = [_Peer("127.0.0.1", hang.getsockname()[1]), _Peer("127.0.0.1", full.port)]
    sched = Scheduler(2, 7, 1.0)
    oracle = OracleLearner("me", ["a", "b"], 1.0, "clock", None, 0.0, 7)
    for r in range(6):
        sched.bernoulli()
        oracle.update_send(1.0)
        res = fetch_loop(sched, peers, 100)
        _, pl, att = oracle.fetch(lambda p: "ok", lambda p: ("timeout", None, None) if p == "a" else
                                  ("payload", {}, b"x"))
        assert res is not None and res[0] == 1
        assert sched.scores() == oracle.scores(["a", "b"]), r
    full.shutdown()
    hang.close()
