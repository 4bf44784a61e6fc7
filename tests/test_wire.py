"""Wire format against the reference's own frames (tests/golden/wire.json, produced by
running dpwa/messaging.py send_message/recv_message over a socketpair).  CPU only."""
import pickle
import socket
import threading

import pytest

from dpwa_amd import wire
from tests.helpers import load_json


def test_constants_match_reference():
    data = load_json("wire.json")
    assert data["header_fmt"] == wire.HEADER_FMT
    assert data["header_len"] == wire.HEADER_LEN
    assert data["chunk_size"] == wire.CHUNK_SIZE


def test_encode_is_byte_identical_to_reference():
    for s in load_json("wire.json")["samples"]:
        payload = None if s["payload_hex"] is None else bytes.fromhex(s["payload_hex"])
        assert wire.encode(s["type"], s["message"], payload).hex() == s["frame_hex"]


def test_decode_reference_frames():
    for s in load_json("wire.json")["samples"]:
        t, m, p = wire.decode(bytes.fromhex(s["frame_hex"]))
        d = s["decoded"]
        assert t == d["type"] and m == d["message"]
        assert (p.hex() if p is not None else None) == d["payload_hex"]


def test_socket_roundtrip_large_payload():
    a, b = socket.socketpair()
    payload = bytes(range(256)) * (3 * 1024 * 1024 // 256 + 7)      # > one 8 MiB chunk? no: ~3 MiB
    payload = payload * 4                                            # ~12 MiB: crosses CHUNK_SIZE
    state = {"clock": 12.5, "loss": 0.25}
    th = threading.Thread(target=wire.send_frame, args=(a, 1, state, payload))
    th.start()
    t, m, p = wire.recv_frame(b)
    th.join()
    assert t == 1 and m == state and p == payload
    a.close()
    b.close()


def test_unsafe_pickle_is_refused():
    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    frame = wire.struct.pack(wire.HEADER_FMT, 1, 0, 0)
    evil = pickle.dumps(Evil())
    frame = wire.struct.pack(wire.HEADER_FMT, 1, len(evil), 0) + evil
    with pytest.raises(pickle.UnpicklingError):
        wire.decode(frame)


def test_closed_connection_raises_message_error():
    a, b = socket.socketpair()
    a.sendall(wire.struct.pack(wire.HEADER_FMT, 1, 0, 100) + b"x" * 10)
    a.close()
    with pytest.raises(wire.MessageError):
        wire.recv_frame(b)
    b.close()


def test_oversize_payload_is_refused():
    class Huge:
        def __len__(self):
            return 1 << 32

    with pytest.raises(wire.MessageError):
        wire.encode(1, None, Huge())


def test_dumps_parts_is_pickle_dumps_with_large_bytes_by_identity():
    """Zero-copy serving: the parts concatenate to pickle.dumps' bytes, and every bytes object of
    64 KiB or more is handed over as itself (so a view of page-locked memory can stand in)."""
    rng = __import__("numpy").random.default_rng(0)
    for sizes in ([10], [100_000], [3, 70_000, 5, 200_000], [0, 1, 65_535, 65_536, 65_537]):
        d = {"p%d" % i: rng.integers(0, 255, s, dtype="uint8").tobytes() for i, s in enumerate(sizes)}
        parts = wire.dumps_parts(d)
        assert b"".join(bytes(p) for p in parts) == pickle.dumps(d)
        big = {id(v) for v in d.values() if len(v) >= 65_536}
        assert {id(p) for p in parts if id(p) in big} == big


def test_param_views_reads_every_protocol_without_copies_and_refuses_the_rest():
    rng = __import__("numpy").random.default_rng(1)
    d = {"w%d" % i: rng.integers(0, 255, s, dtype="uint8").tobytes() for i, s in enumerate([0, 7, 300, 70_000])}
    for proto in (3, 4, 5):
        blob = bytearray(pickle.dumps(d, protocol=proto))
        v = wire.param_views(blob)
        assert {k: bytes(x) for k, x in v.items()} == d
        assert all(x.obj is not None for x in v.values())        # views of `blob`, not copies
        blob[-1] = 0                                              # no STOP: not accepted
        assert wire.param_views(blob) is None
    for other in ({"a": 1}, [b"x"], {1: b"x"}, {"a": {"b": b"x"}}, "s"):
        assert wire.param_views(pickle.dumps(other)) is None


def test_parts_and_receive_into_a_caller_buffer():
    a, b = socket.socketpair()
    big = bytes(range(256)) * 50_000
    parts = [b"head", memoryview(big)[100:], b"tail"]
    state = {"clock": 3, "loss": 0.5}
    th = threading.Thread(target=wire.send_frame_parts, args=(a, 1, state, parts))
    th.start()
    buf = bytearray(len(big) + 64)
    t, m, p = wire.recv_frame_into(b, lambda n: buf)
    th.join()
    assert t == 1 and m == state and bytes(p) == b"head" + big[100:] + b"tail"
    assert p.obj is buf
    a.close()
    b.close()
