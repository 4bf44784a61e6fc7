"""Gossip groups: how a DpwaConnection finds its peers' snapshots.

The reference finds peers by (host, port) from the YAML and fetches over TCP
(dpwa/conn.py:208-213, 246-251, 297-298).  On MI355X a node is a learner on a GPU and a
fetch is a device-to-device pull, so a group answers three questions for the scheduler:
who is up, who has published (the reference's ``have_state``, conn.py:106), and where a
peer's snapshot lives.

``LocalGroup``  every node of the config lives in this process (single-GPU multi-learner
                runs, tests).  A node that has not been constructed yet is "down" (the
                reference's ConnectionRefusedError); one that has not published is
                "no state" (the empty reply).  Fetches are resolved at update_wait, after
                every learner of the round has published (lock-step order).
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

    def join(self, conn):
        old = self.members.get(conn.name)
        if old is not None and old() is not None and old() is not conn:
            raise OSError(98, "node %r is already bound in this process" % conn.name)   # EADDRINUSE
        self.members[conn.name] = weakref.ref(conn)

    def leave(self, conn):
        ref = self.members.get(conn.name)
        if ref is not None and ref() is conn:
            del self.members[conn.name]

    def member(self, name):
        ref = self.members.get(name)
        return ref() if ref is not None else None

    def on_bind(self, conn):
        pass

    def after_publish(self, conn, stream):
        pass

    def peer_status(self, conn, peer_name):
        peer = self.member(peer_name)
        if peer is None:
            return _lib.PEER_DOWN
        if peer._learner is None or peer._learner.version == 0:
            return _lib.PEER_NO_STATE
        return _lib.PEER_READY

    def prepare_fetch(self, conn, peer_index):
        peer = self.member(conn.peers[peer_index].name)
        key = ("local", id(peer._learner))
        if conn._attached.get(peer_index) != key:
            conn._learner.attach_local(peer_index, peer._learner)
            conn._attached[peer_index] = key
        return peer._learner.version, self.zero_copy


class DistGroup:
    """One learner per rank; see the module docstring."""
    eager_fetch = True

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
        self.index = {p.name: i for i, p in enumerate(conn.peers)}

    def leave(self, conn):
        pass

    def on_bind(self, conn):
        """Collective: every rank exports its snapshot allocation and maps every peer's."""
        handle = conn._learner.ipc_handle()
        handles = [None] * self.world
        self.dist.all_gather_object(handles, handle, group=self.pg)
        for k, peer in enumerate(conn.peers):
            r = conn.peer_rank(k)
            conn._learner.attach_ipc(k, handles[r])
            conn._attached[k] = ("ipc", r)

    def barrier(self, device):
        """Stream-ordered on RCCL (the current stream waits; the host does not)."""
        if self.backend == "nccl":
            if self._flag is None or self._flag.device != device:
                self._flag = torch.zeros(1, dtype=torch.int32, device=device)
            self.dist.all_reduce(self._flag, group=self.pg)
        else:
            torch.cuda.current_stream(device).synchronize()
            self.dist.barrier(group=self.pg)

    def after_publish(self, conn, stream):
        # Every peer's publish of this round is complete (and their fetches of the slot we
        # are about to rewrite two rounds from now are ordered before it) once this returns
        # on `stream`.
        self.barrier(conn._learner.device)

    def peer_status(self, conn, peer_name):
        return _lib.PEER_READY

    def prepare_fetch(self, conn, peer_index):
        # lock-step: every rank has published exactly as often as this one
        return conn._learner.version, False


def default_group(config_file, nodes, name):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() == len(nodes) > 1:
        return DistGroup(nodes, name)
    return LocalGroup.for_config(config_file)
