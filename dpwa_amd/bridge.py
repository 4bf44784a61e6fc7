"""Wire bridge: GPU learners that speak the reference's TCP protocol, so they
can gossip with reference CPU nodes (dpwa/conn.py + dpwa/messaging.py) listed in the same
YAML, off-node included.

* ``SnapshotCodec``  flat buffer <-> the reference's blob, ``pickle.dumps({name: raw bytes})``
                     in ``named_parameters()`` order (dpwa/adapters/pytorch.py:17-34, 49-53).
* ``WireServer``     RxThread's role (conn.py:51-172): serves the learner's latest published
                     snapshot, ``send_message(sock, 1, {'clock','loss'}, blob)`` (conn.py:108-110),
                     or an empty reply before the first publish (conn.py:106-107).  One thread
                     per connection instead of one epoll loop, so fetchers are not serialised.
* ``fetch_loop``     TxThread.run for one queue item (conn.py:277-315) over real sockets, with
                     the native scheduler deciding peers and applying the outcomes.
* ``WireConnection`` DpwaConnection whose peers are reached over TCP: the snapshot is read
                     from HBM to serve it, a fetched reply is staged into HBM
                     (dpwa_learner_fetch_host) and averaged by the same fused kernel.

Frames are parsed with a plain-data unpickler (dpwa_amd.wire.safe_loads).  Only float32
parameters can be bridged: the reference maps only FloatTensor (pytorch.py:11-14).
"""
import ctypes
import logging
import socket
import struct
import threading

import numpy as np
import torch

from . import _lib, wire
from .dpwa import DeviceFactor, DpwaConnection, PeerSnapshot

LOGGER = logging.getLogger(__name__)

TCP_SOCKET_BUFFER_SIZE = 8 * 1024 * 1024      # conn.py:40
_PICKLE_FRAME_TARGET = 64 * 1024              # pickle writes bytes objects this large outside its frames


def _tune(sock):
    """conn.py:42-48."""
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, TCP_SOCKET_BUFFER_SIZE)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, TCP_SOCKET_BUFFER_SIZE)
    sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    return sock


class SnapshotCodec:
    """Flat fp32 buffer layout (names, element offsets, numels, total) <-> reference blob."""

    def __init__(self, names, offsets, numels, total):
        self.names, self.offsets, self.numels, self.total = list(names), list(offsets), list(numels), int(total)
        self._placeholders = {}

    @classmethod
    def from_flat(cls, flat):
        """From a dpwa_amd.flat.FlatParameters."""
        return cls(flat.names, flat.offsets, [p.numel() for p in flat.params], flat.numel)

    @classmethod
    def single(cls, name, numel):
        return cls([name], [0], [numel], numel)

    def to_blob(self, payload):
        """payload: bytes of the flat fp32 buffer -> pickle.dumps({name: bytes})."""
        a = np.frombuffer(payload, dtype=np.float32, count=self.total)
        params = {}
        for name, off, n in zip(self.names, self.offsets, self.numels):
            params[name] = a[off:off + n].tobytes()
        import pickle
        return pickle.dumps(params)

    def to_parts(self, payload):
        """payload: a buffer holding the flat fp32 buffer (page-locked host memory, say) -> the
        parts of to_blob's bytes, every parameter of 64 KiB or more as a view of `payload` (no
        copy).  The pickler is run over same-length placeholders (bytes(n) is lazily zeroed
        memory, never touched), which it hands on by identity; each is then swapped for its view."""
        mv = memoryview(payload).cast("B")
        params, swap = {}, {}
        for i, (name, off, n) in enumerate(zip(self.names, self.offsets, self.numels)):
            seg = mv[off * 4:(off + n) * 4]
            if n * 4 >= _PICKLE_FRAME_TARGET:
                ph = self._placeholders.get((i, n))
                if ph is None:
                    ph = self._placeholders[(i, n)] = bytes(n * 4)
                params[name] = ph
                swap[id(ph)] = seg
            else:
                params[name] = bytes(seg)
        return [swap.get(id(p), p) for p in wire.dumps_parts(params)]

    def is_identity(self):
        """One parameter covering the whole flat buffer: a received blob is the flat layout."""
        return len(self.names) == 1 and self.offsets[0] == 0 and self.numels[0] == self.total

    def assemble(self, views, out):
        """{name: buffer} (param_views / safe_loads of a reference blob) -> the flat layout in
        `out` (a float32 array of `total` elements whose gaps stay as they are).  KeyError for a
        missing parameter, like the adapter's other_params[name] (pytorch.py:67)."""
        for name, off, n in zip(self.names, self.offsets, self.numels):
            a = np.frombuffer(views[name], dtype=np.float32)
            if a.size != n:
                raise ValueError("parameter %r has %d elements in the peer's blob, %d here" % (name, a.size, n))
            out[off:off + n] = a

    def from_blob(self, blob):
        """Reference blob -> bytes of the flat layout (gaps zero).  KeyError for a missing
        parameter, like the adapter's other_params[name] (pytorch.py:67)."""
        params = wire.safe_loads(blob)
        out = np.zeros(self.total, dtype=np.float32)
        for name, off, n in zip(self.names, self.offsets, self.numels):
            buf = params[name]
            a = np.frombuffer(buf, dtype=np.float32)
            if a.size != n:
                raise ValueError("parameter %r has %d elements in the peer's blob, %d here" % (name, a.size, n))
            out[off:off + n] = a
        return out.tobytes()


def header_bytes(clock, loss, n, version=1):
    """A dpwa_header (include/dpwa_hip.h) for a snapshot that arrived over the wire."""
    return struct.pack("<ddQqii", float(clock), float(loss), version, n, _lib.F32, 0) + bytes(216)


class WireServer:
    """RxThread (conn.py:51-172) for a GPU learner; ``snapshot_fn() -> (state, blob) | None``, or
    ``(state, parts, release)``: the payload as a list of buffers, and a callable run once they
    have been sent."""

    def __init__(self, host, port, snapshot_fn, timeout_ms):
        self.snapshot_fn = snapshot_fn
        self.timeout = timeout_ms / 1000.0     # the reference's Rx side passes ms as seconds (conn.py:142)
        self.sock = _tune(socket.socket(socket.AF_INET, socket.SOCK_STREAM))
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(64)
        self.port = self.sock.getsockname()[1]
        self._stop = False
        self._threads = []
        self._accept = threading.Thread(target=self._run, daemon=True, name="dpwa-wire-rx-%d" % self.port)
        self._accept.start()

    def _run(self):
        while not self._stop:
            try:
                client, _ = self.sock.accept()
            except OSError:
                break
            client.settimeout(self.timeout)
            t = threading.Thread(target=self._serve, args=(client,), daemon=True)
            t.start()
            self._threads.append(t)

    def _serve(self, client):
        try:
            while not self._stop:
                mtype, _, _ = wire.recv_frame(client)
                if mtype != wire.MESSAGE_TYPE_FETCH_PARAMETERS:
                    raise wire.MessageError("unexpected message type %d" % mtype)
                snap = self.snapshot_fn()
                if snap is None:
                    wire.send_frame(client, wire.MESSAGE_TYPE_FETCH_PARAMETERS)           # conn.py:106-107
                elif len(snap) == 3:      # (state, payload parts, release): views of a pinned buffer
                    try:
                        wire.send_frame_parts(client, wire.MESSAGE_TYPE_FETCH_PARAMETERS, snap[0], snap[1])
                    finally:
                        snap[2]()
                else:
                    wire.send_frame(client, wire.MESSAGE_TYPE_FETCH_PARAMETERS, snap[0], snap[1])
        except (wire.MessageError, OSError) as e:
            LOGGER.debug("wire server: closing connection (%s)", e)
        finally:
            client.close()

    def shutdown(self):
        """Clean shutdown (the reference's RxThread.shutdown raises NotImplementedError)."""
        self._stop = True
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()
        self._accept.join(timeout=5)


class _Peer:
    def __init__(self, host, port):
        self.host, self.port = host, port
        self.sock = None


def fetch_loop(sched, peers, timeout_ms, max_attempts=100000, alloc=None):
    """TxThread.run for one queue item (conn.py:277-315) over real sockets.

    `sched` is the native scheduler (dpwa_amd.sched.Scheduler); `peers` are _Peer objects in
    scheduler order.  Returns (k, state, payload) or None.  alloc(n): where a reply's payload
    is received (wire.recv_frame_into; the payload is then a view of it), else a bytes object."""
    timeout = timeout_ms / 1000.0
    for _ in range(max_attempts):
        k, connected = sched.pick()                      # conn.py:227-240
        if k < 0:
            return None
        p = peers[k]
        if not connected:                                # conn.py:246-260
            try:
                s = _tune(socket.socket(socket.AF_INET, socket.SOCK_STREAM))
                s.settimeout(timeout)
                s.connect((p.host, p.port))
            except ConnectionRefusedError:
                sched.report(k, "refused")
                return None
            except OSError:
                sched.report(k, "connect_error")
                return None
            p.sock = s
            sched.report(k, "connect_ok")
        try:                                             # conn.py:294-313
            wire.send_frame(p.sock, wire.MESSAGE_TYPE_FETCH_PARAMETERS)
            _, state, payload = wire.recv_frame_into(p.sock, alloc) if alloc else wire.recv_frame(p.sock)
        except socket.timeout:
            sched.report(k, "timeout")
            p.sock.close()
            p.sock = None
            continue
        except Exception as e:                           # noqa: BLE001 - the reference removes the peer
            LOGGER.warning("wire fetch from %s:%d failed: %s", p.host, p.port, e)
            sched.report(k, "error")
            p.sock.close()
            p.sock = None
            continue
        done, data = sched.report(k, "payload" if payload is not None else "empty")
        if data:
            return k, state, payload
    return None


class _WireGroup:
    eager_fetch = False      # the fetch is driven by WireConnection itself
    zero_copy = False

    def join(self, conn):
        pass

    def leave(self, conn):
        pass

    def on_bind(self, conn):
        pass

    def after_publish(self, conn):
        pass


class WireConnection(DpwaConnection):
    """DpwaConnection whose peers are reached over TCP at the (host, port) of the YAML.

    eager=True starts the fetch in a background thread at update_send, overlapping the
    training step like the reference's TxThread; eager=False fetches at update_wait
    (deterministic lock-step when every node's update_send precedes every update_wait)."""

    def __init__(self, name, config_file, codec=None, seed=None, eager=True, serve=True):
        super().__init__(name, config_file, seed=seed, group=_WireGroup())
        self.codec = codec
        self.eager = eager
        self._wire_peers = [_Peer(p.host, p.port) for p in self.peers]
        self._thread = None
        self._result = None
        self._averaged_once = False
        # served snapshots: page-locked host copies, each with the frame parts viewing it and
        # the number of replies still sending it (a new version takes a copy nobody is sending)
        self._snap_lock = threading.Lock()
        self._snaps = []
        self._snap_cur = None
        # received replies land in page-locked memory the host-to-device copy reads directly
        self._rx = None
        self._flat_host = None
        self._server = WireServer(self.me.host, self.me.port, self._snapshot, self.timeout_ms) if serve else None

    # -- serving (RxThread) ---------------------------------------------------------
    def _snapshot(self):
        """(state, parts, release) of the newest published snapshot, or None before the first
        publish (conn.py:106-110).  The device copy goes straight to page-locked memory and the
        reply's parameter bytes are views of it (SnapshotCodec.to_parts)."""
        learner = self._learner
        if learner is None:
            return None
        with self._snap_lock:
            cur = self._snap_cur
            if cur is not None and cur["version"] == learner.native_version():
                cur["users"] += 1
                return cur["state"], cur["parts"], lambda e=cur: self._release(e)
            ent = next((e for e in self._snaps if e["users"] == 0 and e is not cur), None)
            if ent is None:
                buf = torch.empty(learner.numel * 4, dtype=torch.uint8, pin_memory=True)
                ent = {"buf": buf, "users": 0, "version": 0}
                self._snaps.append(ent)
            hdr = ctypes.create_string_buffer(256)
            v = ctypes.c_uint64()
            _lib.call("dpwa_learner_read_snapshot", learner.handle, hdr, ctypes.c_void_p(ent["buf"].data_ptr()),
                      learner.numel * 4, ctypes.byref(v))
            if v.value == 0:
                return None
            clock, loss = struct.unpack_from("<dd", hdr.raw)
            if not self._averaged_once and float(clock).is_integer():
                clock = int(clock)       # the reference's clock is an int until the first averaging
            ent.update(version=v.value, state={"clock": clock, "loss": loss},
                       parts=self.codec.to_parts(ent["buf"].numpy()), users=1)
            self._snap_cur = ent
            return ent["state"], ent["parts"], lambda e=ent: self._release(e)

    def _release(self, ent):
        with self._snap_lock:
            ent["users"] -= 1

    def _rx_alloc(self, n):
        if self._rx is None or self._rx.numel() < n:
            self._rx = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        return self._rx.numpy()

    # -- fetching (TxThread) --------------------------------------------------------
    def _fetch(self):
        try:
            self._result = fetch_loop(self._sched, self._wire_peers, self.timeout_ms, alloc=self._rx_alloc)
        except Exception as e:      # noqa: BLE001
            LOGGER.exception("wire fetch failed")
            self._result = e

    def update_send(self, parameters, loss, reuse_snapshot=False):
        if parameters.dtype != torch.float32:
            raise KeyError("the wire bridge carries float32 parameters only (pytorch.py:11-14)")
        self._join()
        super().update_send(parameters, loss, reuse_snapshot)
        self._result = None
        if self.fetching and self.eager:
            self._thread = threading.Thread(target=self._fetch, daemon=True)
            self._thread.start()

    def _join(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def _stage(self):
        """fetch_wait (conn.py:326-329) + staging of the reply into HBM; None for no data."""
        if not self.fetching:
            return None
        self.fetching = False
        if self.eager:
            self._join()
        else:
            self._fetch()
        res = self._result
        self._result = None
        if isinstance(res, Exception):
            raise res
        if res is None:
            return None
        k, state, payload = res
        views = wire.param_views(payload)        # views of the received bytes, no copy
        if views is None:
            views = wire.safe_loads(bytes(payload))   # any other pickle: plain data or an error
        if self.codec.is_identity():             # the blob's one parameter is the flat layout
            src = np.frombuffer(views[self.codec.names[0]], dtype=np.float32)
            if src.size != self.codec.total:
                raise ValueError("parameter %r has %d elements in the peer's blob, %d here"
                                 % (self.codec.names[0], src.size, self.codec.total))
        else:
            if self._flat_host is None:          # gaps between parameters stay zero
                self._flat_host = torch.zeros(self.codec.total, dtype=torch.float32, pin_memory=True).numpy()
            src = self._flat_host
            self.codec.assemble(views, src)
        hdr = header_bytes(state["clock"], state["loss"], self.codec.total)
        learner = self._learner
        # returns once the bytes are on the device side (a page-locked source is waited for),
        # so the receive buffer is free for the next reply
        _lib.call("dpwa_learner_fetch_host", learner.handle, hdr, ctypes.c_void_p(src.ctypes.data), src.nbytes,
                  _lib.stream_handle(torch.cuda.current_stream(learner.device)))
        return k

    def update_wait(self, loss):
        k = self._stage()
        if k is None:
            return None, 0
        self._learner.factor(loss, torch.cuda.current_stream(self._learner.device))
        self._averaged_once = True
        return PeerSnapshot(self, k, 0), DeviceFactor(self._learner)

    def update_wait_average(self, parameters, loss, write_through=False):
        k = self._stage()
        if k is None:
            return None, 0
        stream = torch.cuda.current_stream(self._learner.device)
        if write_through:
            _lib.call("dpwa_learner_average_through", self._learner.handle, parameters.data_ptr(),
                      *self._loss(loss), _lib.stream_handle(stream))
        else:
            self._learner.average(parameters, loss, stream)
        self._averaged_once = True
        return PeerSnapshot(self, k, 0), DeviceFactor(self._learner)

    def _loss(self, loss):
        # the learner's own conversion: it also sets the dtype flag the kernels read a device
        # loss pointer with (a float32 loss tensor is read in place as float32)
        h, d, self._learner._keep = self._learner.loss_args(loss)
        return h, d

    def _bind(self, parameters):
        learner = super()._bind(parameters)
        # served snapshots carry the loss given to update_send (conn.py:110): a write-through
        # average never writes the next header ahead with a placeholder loss
        _lib.call("dpwa_learner_set_header_publish", learner.handle, 1)
        return learner

    @property
    def last_fetch_peer(self):
        return None

    def make_resident(self, parameters):
        raise NotImplementedError("resident parameters need the device transport (the wire bridge reads "
                                  "published slots from the host)")

    def close(self):
        self._join()
        if getattr(self, "_server", None) is not None:
            self._server.shutdown()
            self._server = None
        for p in getattr(self, "_wire_peers", []):
            if p.sock is not None:
                p.sock.close()
                p.sock = None
        super().close()
