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
                GPU per rank.  Snapshot slots are exported with hipIpcGetMemHandle and
                mapped by every peer at the first publish; each round is lock-step: a
                stream-ordered barrier after the publish, then each fetch is pulled over
                xGMI on the learner's side stream while the training step runs.
"""
import os
import threading
import weakref

import torch

from . import _lib


class LocalGroup:
    eager_fetch = False
    zero_copy = True
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

    def __init__(self):
        self.members = {}

    def member(self, name):
        ref = self.members.get(name)
        return ref() if ref is not None else None

    def join(self, conn):
        old = self.member(conn.name)
        if old is not None and old is not conn:
            raise OSError(98, "node %r is already bound in this process" % conn.name)   # EADDRINUSE
        self.members[conn.name] = weakref.ref(conn)
        for k, p in enumerate(conn.peers):          # wire both directions
            other = self.member(p.name)
            if other is None:
                continue
            conn._set_peer(k, _lib.NODE_PEER_LOCAL, other)
            j = other._peer_index.get(conn.name)
            if j is not None:
                other._set_peer(j, _lib.NODE_PEER_LOCAL, conn)

    def leave(self, conn):
        if self.member(conn.name) is not conn:
            return
        del self.members[conn.name]
        for name in list(self.members):
            other = self.member(name)
            j = other._peer_index.get(conn.name) if other is not None else None
            if j is not None:
                other._set_peer(j, _lib.NODE_PEER_UNSET, None)

    def on_bind(self, conn):
        pass

    def after_publish(self, conn):
        pass


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
        self.backend = dist.get_backend(process_group)
        self._flag = None

    def join(self, conn):
        pass

    def leave(self, conn):
        pass

    def on_bind(self, conn):
        """Collective: every rank exports its snapshot allocation and maps every peer's."""
        handle = conn._learner.ipc_handle()
        handles = [None] * self.world
        self.dist.all_gather_object(handles, handle, group=self.pg)
        for k in range(len(conn.peers)):
            conn._learner.attach_ipc(k, handles[conn.peer_rank(k)])
            conn._set_peer(k, _lib.NODE_PEER_REMOTE, None)

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
        # Every peer's publish of this round is complete (and their fetches of the slot we
        # rewrite two rounds from now are ordered before it) once this returns on the stream.
        self.barrier(conn._learner.device)


def default_group(config_file, nodes, name):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() == len(nodes) > 1:
        return DistGroup(nodes, name)
    return LocalGroup.for_config(config_file)
