"""dpwa's TCP wire format (dpwa/messaging.py:9-94), for bridging GPU learners to
reference CPU nodes.

A frame is a 10-byte little-endian header ``<HLL`` = (u16 message type, u32 message
length, u32 payload length), the pickled message (the ``{'clock', 'loss'}`` state dict) and
the raw payload (the pickled ``{name: bytes}`` parameter dict).  ``encode`` produces the
same bytes as the reference's ``send_message``; ``recv_frame`` reads them back with:

* one preallocated buffer filled by ``recv_into`` -- linear in the frame size (the
  reference's ``blob += chunk`` is quadratic, messaging.py:55, minutes at 4 GB);
* a restricted unpickler that only builds plain data (dict, list, tuple, str, bytes,
  numbers, bool, None): frames come from the network, so nothing in them may import or
  call code;
* the reference's u32 limits: a payload of 2**32 bytes or more cannot be framed
  (1B fp32 just fits, 7B bf16 does not -- SURVEY §8 a16).
"""
import io
import pickle
import struct

HEADER_FMT = "<HLL"                 # messaging.py:16
HEADER_LEN = 2 + 4 + 4              # messaging.py:15
CHUNK_SIZE = 8 * (1024 ** 2)        # messaging.py:17
MESSAGE_TYPE_FETCH_PARAMETERS = 1   # conn.py:34
MAX_LEN = 0xFFFFFFFF


class MessageError(Exception):
    """messaging.py:20-21."""


class _PlainDataUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        raise pickle.UnpicklingError("frame refers to %s.%s; only plain data is accepted" % (module, name))


def safe_loads(data):
    """pickle.loads that refuses every global (no code can run)."""
    return _PlainDataUnpickler(io.BytesIO(data)).load()


def encode(message_type, message=None, payload=None):
    """Header + pickle(message) + payload, exactly as send_message builds it (messaging.py:76-88)."""
    message_raw = b"" if message is None else pickle.dumps(message)
    payload = b"" if payload is None else payload
    if len(message_raw) > MAX_LEN or len(payload) > MAX_LEN:
        raise MessageError("frame too large for the <HLL header (%d, %d bytes)" % (len(message_raw), len(payload)))
    return struct.pack(HEADER_FMT, int(message_type), len(message_raw), len(payload)) + message_raw + payload


def send_frame(sock, message_type, message=None, payload=None):
    """messaging.py:76-94, with sendall over memoryview slices (no copies)."""
    hdr_and_msg = encode(message_type, message, None)
    payload = b"" if payload is None else payload
    if len(payload) > MAX_LEN:
        raise MessageError("payload of %d bytes does not fit the u32 length" % len(payload))
    hdr_and_msg = hdr_and_msg[:6] + struct.pack("<L", len(payload)) + hdr_and_msg[HEADER_LEN:]
    sock.sendall(hdr_and_msg)
    mv = memoryview(payload)
    for off in range(0, len(mv), CHUNK_SIZE):
        sock.sendall(mv[off:off + CHUNK_SIZE])


def _recv_exact(sock, buf, n):
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:n], min(CHUNK_SIZE, n - got))
        if k == 0:
            raise MessageError("recv() failed, connection closed. fd={}".format(sock.fileno()))
        got += k


def decode(frame):
    """(type, message, payload) of one complete frame held in memory."""
    if len(frame) < HEADER_LEN:
        raise MessageError("short frame")
    mtype, mlen, plen = struct.unpack(HEADER_FMT, bytes(frame[:HEADER_LEN]))
    if len(frame) != HEADER_LEN + mlen + plen:
        raise MessageError("frame length %d does not match its header (%d)" % (len(frame), HEADER_LEN + mlen + plen))
    message = safe_loads(bytes(frame[HEADER_LEN:HEADER_LEN + mlen])) if mlen else None
    payload = bytes(frame[HEADER_LEN + mlen:]) if plen else None
    return mtype, message, payload


def recv_frame(sock):
    """messaging.py:36-73 semantics: (type, message | None, payload | None)."""
    hdr = bytearray(HEADER_LEN)
    _recv_exact(sock, hdr, HEADER_LEN)
    mtype, mlen, plen = struct.unpack(HEADER_FMT, bytes(hdr))
    body = bytearray(mlen + plen)
    _recv_exact(sock, body, mlen + plen)
    message = safe_loads(bytes(body[:mlen])) if mlen else None
    payload = bytes(body[mlen:]) if plen else None
    return mtype, message, payload
