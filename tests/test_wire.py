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
