"""Gossip groups: how a DpwaConnection's node reaches its peers' snapshots.

The reference finds peers by (host, port) from the YAML and fetches over TCP
(dpwa/conn.py:208-213, 246-251, 297-298).  On MI355X a node is a learner on a GPU and a
fetch is a device-to-device pull; a group only wires the native nodes' peer tables
(dpwa_node_set_peer) -- the per-round logic runs in C++ (dpwa_amd/csrc/node.cpp).

``LocalGroup``  every node of the config lives in this process (single-GPU multi-learner
                runs, tests).  A node that has not been constructed yet is unreachable
                (the reference's ConnectionRefusedError); one that has not published
                answers with no state (the empty reply).  Fetches are resolved at
                update_wait, after every learner of the round has published (lock-step
                order); a same-device peer's slot is read in place (no copy).
``DistGroup``   one node per torch.distributed rank, rank == node index in the YAML, one
                GPU per rank.  Snapshot slots are exported (a hipIpcGetMemHandle, or for
                allocations of 1.5 GiB and more one fd per 1 GiB chunk handed over a Unix
                socket: hipIpcOpenMemHandle does not return above ~2 GiB on this ROCm stack)
                and mapped by every peer at the first publish; each round is lock-step: a
                stream-ordered barrier after the publish, then each fetch is pulled over
                xGMI on the learner's side stream while the training step runs.
``AsyncDistGroup`` the same ranks and pulls in free-running rounds through the gossip board,
                no collective per round (the default under torch.distributed).
"""
import ctypes
import os
import socket
import threading
import weakref

import torch

from . import _lib


def _address(node):
    """(host, port) of a YAML node entry as the reference dials it (conn.py:250); localhost
    and 127.0.0.1 are one address."""
    host = str(getattr(node, "host", ""))
    return ("127.0.0.1" if host == "localhost" else host, int(getattr(node, "port", -1)))


class LocalGroup:
    """prefetch: once every learner of the group has published the round, start all granted
    fetches at once on the learners' side streams, so the pulls overlap the training step that
    follows (worth it when peers live on other GPUs of this process; lock-step semantics are
    unchanged).  zero_copy=False makes same-device fetches copy into staging too."""
    eager_fetch = False
    _registry = {}
    _lock = threading.Lock()

    @classmethod
    def for_config(cls, config_file):
        key = os.path.realpath(config_file)
        with cls._lock:
            g = cls._registry.get(key)
            if g is None:
                g = cls._registry[key] = cls()
            return g

    def __init__(self, prefetch=False, zero_copy=True):
        self.members = {}
        self.prefetch = prefetch
        self.zero_copy = zero_copy

    def member(self, name):
        ref = self.members.get(name)
        return ref() if ref is not None else None

    def _server(self, p):
        """The member whose RxThread a TxThread dialling peer entry `p` reaches: the reference
        connects by (host, port) (conn.py:246-251), so an entry at a member's own address is that
        member whatever its name -- including the dialling node itself (configs[1]'s self-peer:
        a node entry at the learner's own host:port serves its own published snapshot)."""
        other = self.member(p.name)
        if other is not None:
            return other
        for name in list(self.members):
            m = self.member(name)
            if m is not None and _address(m.me) == _address(p):
                return m
        return None

    def join(self, conn):
        old = self.member(conn.name)
        if old is not None and old is not conn:
            raise OSError(98, "node %r is already bound in this process" % conn.name)   # EADDRINUSE
        self.members[conn.name] = weakref.ref(conn)
        for k, p in enumerate(conn.peers):          # wire both directions
            other = self._server(p)
            if other is not None:
                conn._set_peer(k, _lib.NODE_PEER_LOCAL, other)
        for name in list(self.members):
            other = self.member(name)
            if other is None or other is conn:
                continue
            for j, q in enumerate(other.peers):
                if q.name == conn.name or _address(q) == _address(conn.me):
                    other._set_peer(j, _lib.NODE_PEER_LOCAL, conn)

    def leave(self, conn):
        if self.member(conn.name) is not conn:
            return
        del self.members[conn.name]
        for name in list(self.members):
            other = self.member(name)
            if other is None:
                continue
            for j, q in enumerate(other.peers):
                if q.name == conn.name or _address(q) == _address(conn.me):
                    other._set_peer(j, _lib.NODE_PEER_UNSET, None)

    def on_bind(self, conn):
        pass

    def after_publish(self, conn):
        pass

    def after_gate(self, conn):
        pass

    def after_update_send(self, conn):
        if not self.prefetch:
            return
        members = [self.member(n) for n in list(self.members)]
        members = [m for m in members if m is not None]
        if any(m._learner is None for m in members):
            return
        v = conn._learner.version
        if any(m._learner.version != v for m in members):
            return                      # someone has not published this round yet
        for m in members:
            if m.fetching:
                _lib.call("dpwa_node_start_fetch", m._node, m._flags, m._raw_stream(m._learner.device.index))


class _FdServer:
    """Hands this rank's exported chunk fds (SCM_RIGHTS over an abstract Unix socket on this
    host) to each of `expected` peers, then closes them.  Abstract socket names are visible to
    every local user (/proc/net/unix), so a connection is served only if its SO_PEERCRED shows
    this user's uid and the pid of one of the job's ranks (``allow``, after the ranks have
    exchanged pids); any other connection is closed unserved and does not use up a peer's turn."""
    TIMEOUT_S = 600

    def __init__(self, fds, expected):
        if len(fds) > 250:          # one SCM_RIGHTS message carries at most 253 fds
            raise ValueError("%d chunk fds exceed one socket message; allocations this large are not supported"
                             % len(fds))
        self.fds, self.error = list(fds), None
        self.rejected = 0
        self._allowed = None
        self._ready = threading.Event()
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.address = "\0dpwa-fds-%d-%s" % (os.getpid(), os.urandom(8).hex())
        self.sock.bind(self.address)
        self.sock.listen(max(4, expected))
        self.sock.settimeout(self.TIMEOUT_S)
        self.thread = threading.Thread(target=self._serve, args=(expected,), daemon=True)
        self.thread.start()

    def allow(self, pids):
        """The pids that may receive the fds (the peer ranks' processes)."""
        self._allowed = {int(p) for p in pids}
        self._ready.set()

    def _serve(self, expected):
        import struct
        try:
            served = 0
            while served < expected:
                c, _ = self.sock.accept()
                with c:
                    pid, uid, _ = struct.unpack("3i", c.getsockopt(socket.SOL_SOCKET, socket.SO_PEERCRED,
                                                                   struct.calcsize("3i")))
                    if not self._ready.wait(self.TIMEOUT_S):
                        raise TimeoutError("the ranks' pids never arrived")
                    if uid != os.getuid() or pid not in self._allowed:
                        self.rejected += 1
                        continue
                    socket.send_fds(c, [b"dpwa"], self.fds)
                    served += 1
        except Exception as e:      # reported by finish()
            self.error = e

    def abort(self):
        """Stops serving now (the exchange failed elsewhere): no one gets the fds."""
        self._allowed = set()
        self._ready.set()
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()

    def finish(self):
        self.thread.join(self.TIMEOUT_S)
        self.sock.close()
        for fd in self.fds:
            os.close(fd)
        self.fds = []
        if self.thread.is_alive() or self.error is not None:
            raise RuntimeError("handing the snapshot allocation's fds to the peers failed: %r" % (self.error,))


def _fetch_fds(address, n):
    """The `n` fds a peer's _FdServer at `address` hands out."""
    with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
        s.settimeout(_FdServer.TIMEOUT_S)
        s.connect(address)
        _, fds, _, _ = socket.recv_fds(s, 16, n)
    if len(fds) != n:
        for fd in fds:
            os.close(fd)
        raise RuntimeError("expected %d fds from the peer, got %d" % (n, len(fds)))
    return fds


class DistGroup:
    """One learner per rank; see the module docstring."""
    eager_fetch = True
    zero_copy = False

    def __init__(self, nodes, name, process_group=None):
        import torch.distributed as dist
        self.dist = dist
        self.pg = process_group
        self.rank = dist.get_rank(process_group)
        self.world = dist.get_world_size(process_group)
        if self.world != len(nodes):
            raise ValueError("DistGroup: %d nodes in the config but world size %d" % (len(nodes), self.world))
        if nodes[self.rank]["name"] != name:
            raise ValueError("DistGroup: rank %d is node %r in the config, not %r"
                             % (self.rank, nodes[self.rank]["name"], name))
        if not _single_host(dist, process_group):
            raise ValueError("the torch.distributed job spans several hosts: the device transport maps peers' "
                             "snapshot slots over IPC/xGMI within one node only; use "
                             "DpwaPyTorchAdapter(..., transport='wire') (the reference's TCP protocol) across hosts")
        self.backend = dist.get_backend(process_group)
        self._flag = None
        self.relay_blocks = 0        # > 0: relay transport (set by the connection's pull mode)
        self.relay_ready = False     # relay buffers allocated and exchanged
        self.relay_fused = False     # phase 2 read by the averaging kernel itself (pull "relay-avg")
        self._picks = None
        self._pick = None

    def join(self, conn):
        pass

    def leave(self, conn):
        pass

    def on_bind(self, conn):
        """Collective: every rank exports its snapshot allocation and maps every peer's (and,
        for the relay transport, its relay buffer)."""
        learner = conn._learner
        handle = learner.ipc_handle()
        relay = b""
        if self.relay_blocks:
            _lib.call("dpwa_learner_relay_enable", learner._h, self.world, self.rank)
            buf = ctypes.create_string_buffer(_lib.IPC_HANDLE_BYTES)
            _lib.call("dpwa_learner_relay_handle", learner._h, buf, _lib.IPC_HANDLE_BYTES)
            relay = buf.raw
        slot_fds, slot_chunk = learner.export_fds(0)
        relay_fds, relay_chunk = learner.export_fds(1) if self.relay_blocks else ([], 0)
        server = _FdServer(slot_fds + relay_fds, self.world - 1) if (slot_fds or relay_fds) else None
        mine = (handle, relay, server.address if server else None, len(slot_fds), slot_chunk, len(relay_fds),
                relay_chunk, os.getpid())
        infos = [None] * self.world
        try:
            self.dist.all_gather_object(infos, mine, group=self.pg)
            if server is not None:      # only the job's ranks may take our fds
                server.allow(info[7] for r, info in enumerate(infos) if r != self.rank)
            for k in range(len(conn.peers)):
                r = conn.peer_rank(k)
                h, rh, address, ns, cs, nr, cr, _ = infos[r]
                fds = _fetch_fds(address, ns + nr) if address else []
                try:
                    if ns:
                        learner.attach_fds(k, h, fds[:ns], cs)
                    else:
                        learner.attach_ipc(k, h)
                    if self.relay_blocks:
                        blob = ctypes.create_string_buffer(bytes(rh), _lib.IPC_HANDLE_BYTES)
                        if nr:
                            arr = (ctypes.c_int * nr)(*fds[ns:])
                            _lib.call("dpwa_learner_relay_attach_fds", learner._h, r, k, blob, _lib.IPC_HANDLE_BYTES,
                                      arr, nr, cr)
                        else:
                            _lib.call("dpwa_learner_relay_attach", learner._h, r, k, blob, _lib.IPC_HANDLE_BYTES)
                finally:
                    for fd in fds:
                        os.close(fd)
                conn._set_peer(k, _lib.NODE_PEER_REMOTE, None)
        except BaseException:
            if server is not None:      # do not leave the serving thread in accept() for TIMEOUT_S
                server.abort()
                server.thread.join(5)
                for fd in server.fds:
                    os.close(fd)
                server.fds = []
            raise
        else:
            if server is not None:
                server.finish()
        if self.relay_blocks:
            dev = learner.device
            self._pick = torch.full((1,), -1, dtype=torch.int32, device=dev)
            self._picks = torch.full((self.world,), -1, dtype=torch.int32, device=dev)
            side = ctypes.c_void_p()
            _lib.call("dpwa_learner_side_stream", learner._h, ctypes.byref(side))
            self._side = torch.cuda.ExternalStream(side.value, device=dev)
            self.relay_ready = True

    def barrier(self, device):
        """Stream-ordered on RCCL (the current stream waits; the host does not)."""
        if self.backend == "nccl":
            if self._flag is None or self._flag.device != device:
                self._flag = torch.zeros(1, dtype=torch.int32, device=device)
            self.dist.all_reduce(self._flag, group=self.pg)
        else:
            torch.cuda.current_stream(device).synchronize()
            self.dist.barrier(group=self.pg)

    def after_publish(self, conn):
        if self.relay_blocks:
            # the relay's barrier is the pick exchange in after_gate; before it, the stream
            # waits for last round's relay work (its reads of our slot and relay buffer)
            _lib.call("dpwa_learner_relay_wait", conn._learner._h,
                      torch.cuda.current_stream(conn._learner.device).cuda_stream)
            return
        # Every peer's publish of this round is complete (and their fetches of the slot we
        # rewrite two rounds from now are ordered before it) once this returns on the stream.
        self.barrier(conn._learner.device)

    def after_gate(self, conn):
        """Relay transport: share every rank's pick (this is the round's barrier: all
        publishes are complete after it), relay phase 1, a barrier on the side stream,
        phase 2.  Every rank runs this every round, fetching or not."""
        if not self.relay_blocks:
            return
        learner = conn._learner
        dev = learner.device
        k = conn._info()[1] if conn.fetching else -1
        pick = conn.peer_rank(k) if k >= 0 else -1
        version = learner.native_version()
        self._exchange_picks(pick, dev)
        cur = torch.cuda.current_stream(dev).cuda_stream
        _lib.call("dpwa_learner_relay_phase1", learner._h, self._picks.data_ptr(), version,
                  self.relay_blocks, cur)
        self._side_barrier(dev)
        _lib.call("dpwa_learner_relay_phase2", learner._h, self._picks.data_ptr(), pick, version,
                  self.relay_blocks, 1 if self.relay_fused else 0)

    def _exchange_picks(self, pick, dev):
        """Every rank's pick into self._picks (device int32[world]); on RCCL an all-gather ordered
        on the current stream (it is the round's barrier: every publish before it is complete)."""
        if self.backend == "nccl":
            self._pick.fill_(pick)
            self.dist.all_gather_into_tensor(self._picks, self._pick, group=self.pg)
        else:
            torch.cuda.current_stream(dev).synchronize()
            got = [torch.zeros(1, dtype=torch.int32) for _ in range(self.world)]
            self.dist.all_gather(got, torch.tensor([pick], dtype=torch.int32), group=self.pg)
            self._picks.copy_(torch.cat(got))

    def _side_barrier(self, dev):
        """The barrier between the relay's phases, on the side stream (RCCL: stream-ordered, the
        host does not wait)."""
        if self.backend == "nccl":
            with torch.cuda.stream(self._side):
                self._flag_side = getattr(self, "_flag_side", None)
                if self._flag_side is None:
                    self._flag_side = torch.zeros(1, dtype=torch.int32, device=dev)
                self.dist.all_reduce(self._flag_side, group=self.pg)
        else:
            self._side.synchronize()
            self.dist.barrier(group=self.pg)


class AsyncDistGroup(DistGroup):
    """Free-running rounds between the ranks of one node: no barrier, no collective per
    round.  Peers' snapshots are read through a gossip board (dpwa_amd/csrc/board.cpp): a
    shared-memory block holding every rank's newest complete publish and who is reading
    which version, so a publish waits only for readers of the snapshot it would rewrite --
    the reference's RxThread Lock (conn.py:76-79, 109-110) -- and a rank that has closed or
    died answers as a refused connection (conn.py:253-256).  The copy and kernel pulls and
    write-through snapshots are supported; the relay needs lock-step rounds."""

    def __init__(self, nodes, name, process_group=None, publish_timeout_ms=None):
        super().__init__(nodes, name, process_group)
        self.board = None
        # a publish waits for a slow reader at most this long (the reference blocks forever)
        self.publish_timeout_ms = int(publish_timeout_ms if publish_timeout_ms is not None else 600_000)

    def on_bind(self, conn):
        if getattr(conn, "_pull", "copy").partition(":")[0] in ("relay", "relay-avg") or self.relay_blocks:
            raise ValueError("the relay pull needs lock-step rounds (DistGroup), not free-running ones")
        board = ctypes.c_void_p()
        bname = None
        if self.rank == 0:
            bname = "/dpwa_board_%d_%s" % (os.getpid(), os.urandom(4).hex())
            _lib.call("dpwa_board_open", ctypes.byref(board), bname.encode(), self.world, 0, 1)
        names = [None] * self.world
        self.dist.all_gather_object(names, bname, group=self.pg)     # rank 0 created it
        bname = names[0]
        if self.rank != 0:
            _lib.call("dpwa_board_open", ctypes.byref(board), bname.encode(), self.world, self.rank, 0)
        self.board = board
        _lib.call("dpwa_board_register", board, conn._learner.device.index)
        super().on_bind(conn)                 # IPC exchange; a collective, so every rank has opened
        if self.rank == 0:
            _lib.call("dpwa_board_unlink", bname.encode())   # nothing left in /dev/shm after a crash
        ranks = (ctypes.c_int32 * max(1, len(conn.peers)))(*[conn.peer_rank(k) for k in range(len(conn.peers))])
        _lib.call("dpwa_node_set_board", conn._node, board, ranks, self.publish_timeout_ms)

    def after_publish(self, conn):
        pass

    def after_gate(self, conn):
        pass

    def leave(self, conn):
        board, self.board = self.board, None
        if board is not None and board.value:
            if conn._node is not None and conn._node.value:
                _lib.call("dpwa_node_set_board", conn._node, None, None, -1)
            if conn._learner is not None:
                torch.cuda.synchronize(conn._learner.device)   # our pulls are done with every peer
            _lib.call("dpwa_board_close", board)


def _single_host(dist, process_group=None):
    """Every rank of the group runs on this host (the IPC/xGMI groups map peers' HBM with
    hipIpcOpenMemHandle, which only works within one node).  torchrun says so through
    LOCAL_WORLD_SIZE; otherwise the ranks compare host identities (a collective)."""
    world = dist.get_world_size(process_group)
    lws = os.environ.get("LOCAL_WORLD_SIZE")
    if process_group is None and lws is not None and os.environ.get("WORLD_SIZE") == str(world):
        return int(lws) == world
    import socket
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            ident = socket.gethostname() + "/" + f.read().strip()
    except OSError:
        ident = socket.gethostname()
    ids = [None] * world
    dist.all_gather_object(ids, ident, group=process_group)
    return len(set(ids)) == 1


def default_group(config_file, nodes, name, gossip=None):
    """LocalGroup when this process holds every node; under torch.distributed with one rank
    per node of the config on one host, free-running rounds (AsyncDistGroup: the reference's
    learners never wait for each other, conn.py:73-79, 98-110) unless `gossip` -- the
    config's optional `- gossip:` key, else $DPWA_GOSSIP -- says "lockstep" (DistGroup:
    deterministic rounds behind a barrier; needed by the relay pull).  A multi-host job
    cannot map peers' HBM: it must use the reference's TCP protocol (transport='wire')."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() == len(nodes) > 1:
        mode = gossip or os.environ.get("DPWA_GOSSIP") or "async"
        if mode not in ("async", "lockstep"):
            raise ValueError("gossip must be 'async' or 'lockstep', got %r" % (mode,))
        return AsyncDistGroup(nodes, name) if mode == "async" else DistGroup(nodes, name)
    return LocalGroup.for_config(config_file)
