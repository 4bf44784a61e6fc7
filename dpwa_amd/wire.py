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
    send_frame_parts(sock, message_type, message, [] if payload is None else [payload])


def send_frame_parts(sock, message_type, message, parts):
    """send_frame whose payload is the concatenation of `parts` (bytes-like objects, e.g. the
    pieces of dumps_parts with views of page-locked memory in them): nothing is joined."""
    views = [memoryview(p).cast("B") for p in parts]
    plen = sum(len(v) for v in views)
    if plen > MAX_LEN:
        raise MessageError("payload of %d bytes does not fit the u32 length" % plen)
    hdr_and_msg = encode(message_type, message, None)
    sock.sendall(hdr_and_msg[:6] + struct.pack("<L", plen) + hdr_and_msg[HEADER_LEN:])
    for mv in views:
        for off in range(0, len(mv), CHUNK_SIZE):
            sock.sendall(mv[off:off + CHUNK_SIZE])


class _PartsWriter:
    """File object for pickle.Pickler that keeps every write as its own part: the pickler hands
    a large bytes object to write() itself, outside any frame, so it is never copied."""

    def __init__(self):
        self.parts = []

    def write(self, b):
        self.parts.append(b)
        return len(b)


def dumps_parts(obj):
    """pickle.dumps(obj) as a list of parts whose concatenation is exactly those bytes (large
    bytes objects inside `obj` appear as parts by identity)."""
    w = _PartsWriter()
    pickle.Pickler(w, protocol=pickle.DEFAULT_PROTOCOL).dump(obj)
    return w.parts


def param_views(blob):
    """The reference's parameter blob, a pickled {str: bytes} dict, as {name: memoryview into
    `blob`} without copying any parameter bytes: the pickle opcodes are walked, accepting only
    what pickling such a dict produces (protocols 3-5).  None for any other stream (the caller
    then falls back to safe_loads, which raises on what it refuses)."""
    mv = memoryview(blob).cast("B")
    n = len(mv)
    pos = 0
    stack, marks, memo = [], [], {}

    def u(k):
        nonlocal pos
        v = int.from_bytes(mv[pos:pos + k], "little")
        pos += k
        return v

    def take(k):
        nonlocal pos
        if k < 0 or pos + k > n:
            raise ValueError("truncated")
        v = mv[pos:pos + k]
        pos += k
        return v

    try:
        while pos < n:
            op = mv[pos]
            pos += 1
            if op == 0x80:                      # PROTO
                pos += 1
            elif op == 0x95:                    # FRAME (a length hint)
                pos += 8
            elif op == 0x7D:                    # EMPTY_DICT
                stack.append({})
            elif op == 0x94:                    # MEMOIZE
                memo[len(memo)] = stack[-1]
            elif op == 0x71:                    # BINPUT
                memo[u(1)] = stack[-1]
            elif op == 0x72:                    # LONG_BINPUT
                memo[u(4)] = stack[-1]
            elif op == 0x68:                    # BINGET
                stack.append(memo[u(1)])
            elif op == 0x6A:                    # LONG_BINGET
                stack.append(memo[u(4)])
            elif op == 0x28:                    # MARK
                marks.append(len(stack))
            elif op in (0x8C, 0x58, 0x8D):      # SHORT_BINUNICODE, BINUNICODE, BINUNICODE8
                stack.append(str(take(u({0x8C: 1, 0x58: 4, 0x8D: 8}[op])), "utf-8"))
            elif op in (0x43, 0x42, 0x8E):      # SHORT_BINBYTES, BINBYTES, BINBYTES8
                stack.append(take(u({0x43: 1, 0x42: 4, 0x8E: 8}[op])))
            elif op == 0x73:                    # SETITEM
                v = stack.pop()
                k = stack.pop()
                if not isinstance(stack[-1], dict) or not isinstance(k, str):
                    return None
                stack[-1][k] = v
            elif op == 0x75:                    # SETITEMS
                m = marks.pop()
                items = stack[m:]
                del stack[m:]
                d = stack[-1]
                if not isinstance(d, dict) or len(items) % 2:
                    return None
                for k, v in zip(items[::2], items[1::2]):
                    if not isinstance(k, str):
                        return None
                    d[k] = v
            elif op == 0x2E:                    # STOP
                out = stack.pop()
                if pos != n or stack or not isinstance(out, dict) or \
                        not all(isinstance(v, memoryview) for v in out.values()):
                    return None
                return out
            else:
                return None
    except (IndexError, KeyError, ValueError, UnicodeDecodeError):
        return None
    return None


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


def recv_frame_into(sock, alloc):
    """recv_frame whose payload lands in alloc(n) -- a writable buffer of at least n bytes (for
    instance page-locked memory the next host-to-device copy reads directly) -- and is
    returned as a memoryview of it, not copied again."""
    hdr = bytearray(HEADER_LEN)
    _recv_exact(sock, hdr, HEADER_LEN)
    mtype, mlen, plen = struct.unpack(HEADER_FMT, bytes(hdr))
    msg = bytearray(mlen)
    _recv_exact(sock, msg, mlen)
    message = safe_loads(bytes(msg)) if mlen else None
    if not plen:
        return mtype, message, None
    view = memoryview(alloc(plen)).cast("B")[:plen]
    _recv_exact(sock, view, plen)
    return mtype, message, view


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
