"""DpwaPyTorchAdapter on MI355X (mirror of dpwa/adapters/pytorch.py).

Same constructor and methods.  Instead of pickling every parameter through the host
(pytorch.py:17-34, 49-53) and averaging tensor by tensor with three ATen kernels and
three temporaries each (pytorch.py:66-68), the parameters live in one flat HBM buffer
(dpwa_amd/flat.py); update_send publishes it with one kernel and update_wait averages it
in place with one fused HIP kernel whose coefficients come from the device factor.

Differences that are intentional: the average is written in place (the reference
rebinds ``param.data`` to a new tensor), and float32 *and* bfloat16 models are accepted
(the reference maps only FloatTensor, pytorch.py:11-14).
"""
import ctypes
import logging

import torch

from .. import _lib
from ..dpwa import DpwaConfiguration, DpwaConnection
from ..flat import FlatParameters

LOGGER = logging.getLogger(__name__)


class DpwaPyTorchAdapter:
    """write_through (extension, default on): the averaging kernel also writes the next
    snapshot, and the next update_send publishes only the header when nothing was modified in
    between -- 4*N*s bytes for the averaging and the publish instead of 5*N*s.  The reference
    loop never touches the parameters between update_wait and the next update_send (README.md
    and examples/pytorch-cifar/main.py:130-145: update_send, forward/backward/step, update_wait).
    Before reusing a snapshot the adapter checks that no parameter was re-homed
    (``param.data = ...``), that no parameter's version counter moved (optimizer steps,
    ``param.add_``, ``load_state_dict``) and that the flat buffer's own counter did not move;
    any of these forces a full publish.  In-place writes through ``param.data`` bypass version
    counters; for them the reuse guard (``reuse_guard``, on by default) compares 4096 16-byte
    words spread over the parameters with the snapshot on the device and publishes in full when
    any differs (two small kernels per update_send, no host sync).  The sampled words move on by
    one each publish, so every word is compared once in any ceil(N*s/16/4095) publishes: a sparse
    write that one publish's samples miss is published late (by a later publish that samples it),
    not never.  A loop that writes parameters sparsely through ``param.data`` between update_wait
    and update_send and needs every snapshot exact should pass ``write_through=False``.

    resident (extension, off by default): the parameters live in the learner's own two snapshot
    slots (``DpwaConnection.make_resident``) and every ``param.data`` is re-pointed to the slot
    they are in after each update_send and update_wait -- a publish moves no bytes and an
    average moves 3*N*s (the write-through form 4*N*s), for one ``.data`` assignment per
    parameter per round on the host.  Writes through ``param.data`` are then always part of the
    next snapshot (no snapshot-reuse check is needed).  The price is the loop order: between update_send
    and update_wait the parameters ARE the snapshot peers read, so nothing may write them
    there.  The reference's loop trains exactly there (README.md:18-29,
    examples/pytorch-cifar/main.py:130-145: update_send, step, update_wait) and keeps the
    default write-through form; a resident adapter needs update_send, update_wait, step (each
    step then comes after the round's average instead of before it).  update_wait raises
    DpwaError when a parameter's (or the flat buffer's) version counter moved since update_send
    -- an optimizer step, ``param.add_``, ``load_state_dict`` in the window.  Writes through
    ``param.data`` bypass version counters; for them the reuse guard (``reuse_guard``) is a window
    guard here: every update_send runs one small kernel that compares the parameters published at
    the previous update_send with 4096 words sampled then, and samples the new ones (no host
    wait); a window found written makes a later update_send (the first that sees the device's
    count) raise DpwaError without publishing (``window_guard_hits`` counts them, checking the last
    check).  The sampled words move on by one each publish (as the reuse guard's), so a sparse write
    repeated every window is caught within ceil(N*s/16/4095) windows.  Code that keeps raw data
    pointers of the parameters across rounds (a captured HIP graph of the training step) must
    not use it."""

    def __init__(self, net, name, config_file, write_through=True, transport="device", reuse_guard=True,
                 resident=False, **connection_kwargs):
        """transport: "device" (peers are learners of this process or of the torch.distributed
        job, pulled from HBM/over xGMI) or "wire" (peers are reached over TCP at the YAML's
        host/port with the reference's protocol -- e.g. reference CPU nodes; dpwa_amd/bridge.py)."""
        if resident and transport != "device":
            raise ValueError("resident parameters need the device transport")
        self._net = net
        gpu = DpwaConfiguration(config_file).get_gpu(name)      # optional per-node placement
        self._flat = FlatParameters(net.named_parameters(), device=None if gpu is None else torch.device("cuda", gpu))
        if transport == "wire":
            from ..bridge import SnapshotCodec, WireConnection
            self._conn = WireConnection(name, config_file, codec=SnapshotCodec.from_flat(self._flat),
                                        **connection_kwargs)
        elif transport == "device":
            self._conn = DpwaConnection(name, config_file, **connection_kwargs)
        else:
            raise ValueError("transport must be 'device' or 'wire'")
        self._write_through = bool(write_through) and transport == "device"
        self._resident = bool(resident)
        self._reuse_guard = bool(reuse_guard)
        self._guard_set = False
        self._versions = None
        self._sent = None           # resident: the version counters at the last update_send
        self._warned_rehome = False

    def _warn_rehome(self, moved):
        """Once per adapter: the caller re-homed a parameter (``param.data = ...``), so its loop
        works on ``param.data`` -- and in-place writes through ``.data`` move no version counter.
        When the device reuse guard has not caught any such write so far (its sampled words all
        matched), say plainly where write-through snapshots can go stale (this re-home itself is
        seen: this round publishes in full).  Reading the guard's count synchronises the device,
        once."""
        self._warned_rehome = True
        hits = self.reuse_guard_hits if self._reuse_guard else 0
        if hits == 0:
            LOGGER.warning(
                "DpwaPyTorchAdapter(%s): %d parameter(s) were re-homed through param.data. Write-through "
                "snapshots (the default) are reused when no version counter moved; in-place writes through "
                "param.data move none and are caught only if they change one of the %d words the reuse guard "
                "samples at that publish (the samples move on by one word per publish). A loop that writes parameters sparsely through param.data between update_wait and "
                "update_send must pass write_through=False, or peers may average with a snapshot that lacks "
                "those writes.", self._conn.name, moved, 4096)

    def _param_versions(self):
        return [p._version for p in self._flat.params] + [self._flat.buffer._version]

    def _check_window(self):
        """Resident form: nothing may have written the parameters since update_send (they are
        the snapshot peers read until the average)."""
        if self._sent is not None and self._param_versions() != self._sent:
            raise _lib.DpwaError(
                "DpwaPyTorchAdapter.update_wait", _lib.ERR_STATE,
                "the parameters were modified between update_send and update_wait (an optimizer step?); "
                "with resident=True they are the snapshot peers read in that window, so the loop must run "
                "update_send -> update_wait -> step.  The reference's order update_send -> step -> "
                "update_wait (README.md, main.py:130-145) needs resident=False (the write-through default)")

    def update_send(self, loss):
        """pytorch.py:42-53: publish the parameters and maybe start a fetch."""
        if _lib.TRACE:
            with _lib.trace_range("adapter.update_send"):
                return self._update_send(loss)
        return self._update_send(loss)

    def _update_send(self, loss):
        if self._resident:
            if self._conn.parameters is None:          # first round: into the learner's slot 0
                self._flat.resync()
                self._flat.rehome(self._conn.make_resident(self._flat.buffer))
                if self._reuse_guard:                      # the window guard (see the class doc)
                    _lib.call("dpwa_learner_set_reuse_guard", self._conn._learner.handle, 1)
            self._flat.resync()                        # a parameter re-homed by the caller
            self._conn.update_send(self._flat.buffer, loss)
            # a publish with no average since the last one moved the parameters into the slot it
            # published (dpwa_learner_relocate): the views follow them
            self._flat.rehome(self._conn.parameters)
            self._sent = self._param_versions()
            return
        moved = self._flat.resync()
        if moved and self._write_through and not self._warned_rehome:
            self._warn_rehome(moved)
        reuse = (self._write_through and moved == 0 and self._versions is not None
                 and self._versions == self._param_versions())
        self._versions = None
        self._conn.update_send(self._flat.buffer, loss, reuse_snapshot=reuse)
        if self._write_through and self._reuse_guard and not self._guard_set:    # bound by now
            _lib.call("dpwa_learner_set_reuse_guard", self._conn._learner.handle, 1)
            self._guard_set = True

    def update_wait(self, loss):
        """pytorch.py:55-68: wait for the fetch and average in place (resident: into the other
        slot, where the parameters are re-pointed)."""
        if _lib.TRACE:
            with _lib.trace_range("adapter.update_wait"):
                return self._update_wait(loss)
        return self._update_wait(loss)

    def _update_wait(self, loss):
        if self._resident:
            if self._conn.parameters is None:         # no update_send yet: nothing to average
                return
            self._check_window()
            self._conn.update_wait_average(self._flat.buffer, loss)
            self._flat.rehome(self._conn.parameters)
            self._sent = None
            return
        payload, _ = self._conn.update_wait_average(self._flat.buffer, loss, write_through=self._write_through)
        if self._write_through and payload is not None:
            self._versions = self._param_versions()

    # -- extensions -------------------------------------------------------------------
    @staticmethod
    def update_wait_many(adapters, losses):
        """update_wait of several adapters whose models share a GPU (co-resident learners of
        one process), in order, with their averages as one dispatch (same results as calling
        update_wait on each)."""
        adapters = list(adapters)
        if not adapters:
            return
        wts = {(a._write_through, a._resident) for a in adapters}
        if len(wts) != 1 or any(not isinstance(a._conn, DpwaConnection) or type(a._conn) is not DpwaConnection
                                for a in adapters):
            for a, loss in zip(adapters, losses):     # mixed forms or wire peers: one by one
                a.update_wait(loss)
            return
        wt, resident = wts.pop()
        if resident:
            for a in adapters:
                a._check_window()
        res = DpwaConnection.update_wait_average_many([a._conn for a in adapters],
                                                      [a._flat.buffer for a in adapters], list(losses),
                                                      write_through=wt)
        for a, (payload, _) in zip(adapters, res):
            if resident and a._conn.parameters is not None:
                a._flat.rehome(a._conn.parameters)
                a._sent = None
            elif wt and payload is not None:
                a._versions = a._param_versions()

    def state_dict(self):
        """The connection's gossip state (clock, scheduler) for a checkpoint beside the model's
        (extension: the reference checkpoints the net but restarts dpwa's clock at 0)."""
        return self._conn.state_dict()

    def load_state_dict(self, state):
        self._conn.load_state_dict(state)

    @property
    def reuse_guard_hits(self):
        """Publishes whose reuse guard found the parameters changed behind the version counters
        (synchronises the device; 0 before the first publish)."""
        if self._conn._learner is None:
            return 0
        hits = ctypes.c_uint32()
        _lib.call("dpwa_learner_reuse_guard_hits", self._conn._learner.handle, ctypes.byref(hits))
        return hits.value

    @property
    def window_guard_hits(self):
        """Resident form: rounds whose parameters the window guard found written between
        update_send and update_wait (waits for the last check; 0 before the first publish)."""
        if self._conn._learner is None:
            return 0
        hits = ctypes.c_uint32()
        _lib.call("dpwa_learner_window_hits", self._conn._learner.handle, ctypes.byref(hits))
        return hits.value

    @property
    def connection(self):
        return self._conn

    @property
    def flat(self):
        return self._flat
