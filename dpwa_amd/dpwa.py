"""DpwaConnection and DpwaConfiguration on MI355X (mirror of dpwa/dpwa.py).

Same names, YAML schema, constructor arguments, ``update_send`` / ``update_wait``
protocol and error behaviour as the reference.  What moves:

* the parameters are a device tensor (the flat buffer), not a pickled blob, and the
  snapshot is a slot in HBM published by a kernel (dpwa/dpwa.py:115-116);
* the clock lives on the GPU; the factor and the new clock are computed there
  (dpwa.py:139-155) and never round-trip through the host;
* TxThread's peer choice / flow control runs in the C++ scheduler with the reference's
  exact random draws (dpwa_amd/sched.py); the fetch is a device-to-device pull;
* a ZeroDivisionError of the interpolation (dpwa.py:143) is detected on the device and
  raised at the next call (or at :meth:`synchronize`), because raising at the call itself
  would need a host sync every round.
"""
import ctypes
import logging
import os

import torch
import yaml

from . import _lib
from .group import default_group
from .interpolation import INTERPOLATION_METHODS
from .learner import DTYPES, Learner, loss_args
from .sched import Scheduler, seed_key

LOGGER = logging.getLogger(__name__)
RELAY_PULLS = ("relay", "relay-avg")   # DistGroup's multi-link transports (dpwa_amd/group.py)
_MANY_CALLS = {}    # update_wait_average_many: argument arrays per set of nodes


class Struct:
    def __init__(self, **entries):
        self.__dict__.update(entries)

    def __repr__(self):
        return 'Struct: ' + repr(self.__dict__)


class DpwaConfiguration:
    """dpwa.py:29-51.  The YAML is a list of single-key maps flattened into a dict.

    The reference calls ``yaml.load(f)`` without a Loader, which raises TypeError on
    PyYAML >= 6; the same documents are read here with the safe loader."""

    def __init__(self, config_file):
        with open(config_file, 'rt') as f:
            self.yaml = yaml.safe_load(f)
        self.config = {}
        for c in self.yaml:
            k = list(c.keys())[0]
            self.config[k] = c[k]

    def get_nodes(self):
        return self.config['nodes']

    def get_interpolation(self):
        interpolation = self.config['interpolation']
        return (interpolation, self.config[interpolation])

    def get_timeoutms(self):
        return self.config['timeout_ms']

    def get_fetch_probability(self):
        return self.config['fetch_probability']

    def get_divergence_threshold(self):
        return self.config['divergence_threshold']

    # -- extensions (absent keys keep the reference behaviour) ------------------------
    def get_gpu(self, name):
        """Per-node `gpu:` key (the device index the node's learner runs on), else None.  The
        reference ignores unknown node keys (dpwa.py:66-72 turns each node into a Struct), so
        a config carrying them still loads there."""
        for node in self.get_nodes():
            if node.get('name') == name and 'gpu' in node:
                return int(node['gpu'])
        return None

    def get_seed(self, name):
        """Per-node `seed:` key, else a top-level `- seed:` entry, else None (OS entropy,
        as the reference, which never seeds `random`)."""
        for node in self.get_nodes():
            if node.get('name') == name and 'seed' in node:
                return node['seed']
        return self.config.get('seed')


class PeerSnapshot:
    """What update_wait returns in place of the reference's pickled payload bytes: the
    fetched snapshot, resident on the learner's GPU.  ``tensor()`` materialises it (a
    stream-ordered device copy) for callers that do the reference adapter's arithmetic
    themselves (pytorch.py:64-68); it is valid until the fetch is averaged or abandoned."""

    def __init__(self, conn, peer_index, version):
        self.peer = conn.peers[peer_index].name
        self.version = version
        self.numel = conn._learner.numel
        self.dtype = conn._learner.dtype
        self._learner = conn._learner
        self._round = conn._learner.version

    def tensor(self):
        learner = self._learner
        if learner._h is None or learner.version != self._round:
            raise RuntimeError("this snapshot's fetch is no longer in flight (a later update_send started a new one)")
        out = torch.empty(self.numel, dtype=self.dtype, device=learner.device)
        _lib.call("dpwa_learner_copy_fetched", learner.handle, ctypes.c_void_p(out.data_ptr()),
                  ctypes.c_void_p(torch.cuda.current_stream(learner.device).cuda_stream))
        return out

    def __repr__(self):
        return "PeerSnapshot(peer=%r, version=%d, numel=%d, dtype=%s)" % (self.peer, self.version, self.numel,
                                                                          self.dtype)


class DeviceFactor:
    """The interpolation factor of dpwa.py:143-147, computed on the device.

    It stands in for the Python float the reference returns (dpwa.py:156), so the adapter's
    statement ``factor * t + (1 - factor) * param`` (pytorch.py:68) works unchanged: in
    arithmetic it becomes a 0-d float64 tensor on the learner's device, copied from the
    coefficient block in stream order (no host sync).  ``1 - factor`` is then computed in
    float64 and each product rounds the scalar to the tensor's dtype, exactly as ATen treats
    the reference's Python float.  ``float(f)`` synchronises and returns the exact double."""

    def __init__(self, learner):
        self._learner = learner
        self._round = learner.version
        self._t = None

    def _check(self):
        learner = self._learner
        if learner._h is None or learner.version != self._round:
            raise RuntimeError("stale factor: a later update_send has started a new round")
        return learner

    def tensor(self):
        if self._t is None:
            learner = self._check()
            t = torch.empty((), dtype=torch.float64, device=learner.device)
            _lib.call("dpwa_learner_copy_factor", learner.handle, ctypes.c_void_p(t.data_ptr()),
                      ctypes.c_void_p(torch.cuda.current_stream(learner.device).cuda_stream))
            self._t = t
        return self._t

    def __float__(self):
        if self._t is not None:
            return float(self._t.item())
        return float(self._check().read_coef().factor)

    def __mul__(self, other):
        return self.tensor() * other

    def __rmul__(self, other):
        return other * self.tensor()

    def __add__(self, other):
        return self.tensor() + other

    def __radd__(self, other):
        return other + self.tensor()

    def __sub__(self, other):
        return self.tensor() - other

    def __rsub__(self, other):
        return other - self.tensor()

    def __truediv__(self, other):
        return self.tensor() / other

    def __rtruediv__(self, other):
        return other / self.tensor()

    def __neg__(self):
        return -self.tensor()

    def coefficients(self):
        c = self._check().read_coef()
        return {"factor": c.factor, "new_clock": c.new_clock, "a": c.a, "b": c.b, "status": c.status}

    def __repr__(self):
        return "DeviceFactor(%r)" % float(self)


class DpwaConnection:
    def __init__(self, name, config_file, seed=None, group=None, pull=None):
        self.name = name
        self.config = DpwaConfiguration(config_file)
        self.nodes = self.config.get_nodes()
        self.fetch_probability = self.config.get_fetch_probability()
        self.fetching = False

        # Initialize the list of peers (dpwa.py:65-72)
        self.peers = []
        self._peer_node_index = []
        for i, node in enumerate(self.nodes):
            node = Struct(**node)
            if node.name == name:
                self.me = node
            else:
                self.peers += [node]
                self._peer_node_index.append(i)
        self.me   # AttributeError for a name that is not in the config, as the reference
        self._peer_index = {p.name: k for k, p in enumerate(self.peers)}
        self._peer_wiring = [(0, None)] * len(self.peers)     # (DPWA_NODE_PEER_*, serving node) per peer

        # Interpolation method (dpwa.py:75-80)
        interpolation_method, interpolation_config = self.config.get_interpolation()
        LOGGER.debug("Using %s interpolation method", interpolation_method)
        if interpolation_config == 0:
            interpolation_config = {}
        self.interpolation = INTERPOLATION_METHODS[interpolation_method](**interpolation_config)
        self.divergence_threshold = self.config.get_divergence_threshold()
        self.timeout_ms = self.config.get_timeoutms()

        # The native node: TxThread's scheduler (conn.py:197-334) + the learner, bound at
        # the first update_send (the reference's connection never sees the model either).
        if seed is None:
            seed = self.config.get_seed(name)
        lib = _lib.load()
        self._lib = lib
        self._node = ctypes.c_void_p()
        cfg = self.interpolation.device_config(self.divergence_threshold)
        if seed is None:
            _lib.call("dpwa_node_create", ctypes.byref(self._node), len(self.peers), None, -1,
                      float(self.fetch_probability), ctypes.byref(cfg))
        else:
            key = seed_key(seed)
            arr = (ctypes.c_uint32 * max(1, len(key)))(*key)
            _lib.call("dpwa_node_create", ctypes.byref(self._node), len(self.peers), arr, len(key),
                      float(self.fetch_probability), ctypes.byref(cfg))
        # the YAML's socket timeout (conn.py:249) judges the device path's pulls (dpwa_node_set_timeout)
        _lib.call("dpwa_node_set_timeout", self._node, int(self.timeout_ms) if self.timeout_ms is not None else -1)
        sched = ctypes.c_void_p()
        _lib.call("dpwa_node_handles", self._node, None, ctypes.byref(sched))
        self._sched = Scheduler(len(self.peers), handle=sched.value)
        self._learner = None
        self._pending_clock = None        # load_state_dict before the learner exists
        self._resident = False      # make_resident was called
        self._sent = None           # resident: (parameters tensor, its version) at update_send
        # transport of copying fetches: "copy" (hipMemcpyAsync) or "kernel[:blocks]"
        self._pull = pull if pull is not None else os.environ.get("DPWA_PULL", "copy")
        self._out = ctypes.c_int()
        self._out_ref = ctypes.byref(self._out)
        self._f_update_send = lib.dpwa_node_update_send
        self._f_publish = lib.dpwa_node_publish
        self._f_gate = lib.dpwa_node_gate
        self._f_wait = lib.dpwa_node_update_wait
        self._f_wait_avg = lib.dpwa_node_update_wait_average
        self._f_lerp = lib.dpwa_node_lerp
        self._raw_stream = torch._C._cuda_getCurrentRawStream
        if group == "async":    # free-running rounds between ranks (gossip board), see group.py
            from .group import AsyncDistGroup
            group = AsyncDistGroup(self.nodes, name)
        elif group == "lockstep":
            from .group import DistGroup
            group = DistGroup(self.nodes, name)
        self._group = group if group is not None else default_group(config_file, self.nodes, name,
                                                                    self.config.config.get("gossip"))
        self._eager = bool(self._group.eager_fetch)
        self._flags = (_lib.FLAG_EAGER if self._group.eager_fetch else 0) | \
                      (_lib.FLAG_ZERO_COPY if self._group.zero_copy else 0)
        self._group.join(self)

    # ---------------------------------------------------------------- reference API
    def add_peer(self, name, host, port):
        """dpwa.py:95-96 -> TxThread.add_peer (conn.py:208-213): the peer gets a fresh record
        (flow-control score 1000, not connected); a removed peer is picked again, after the
        others in pick order, as a re-inserted dict key is.  On MI355X a peer is reached through
        the group, so `name` must be a node of the config (host/port are the reference's
        addressing and are kept only for the call's shape); unknown names raise KeyError."""
        k = self._peer_by_name(name)
        self._sched.add(k)

    def remove_peer(self, name):
        """dpwa.py:98-99 -> TxThread.remove_peer (conn.py:215-222): permanent."""
        _lib.call("dpwa_sched_remove", self._sched._h, self._peer_by_name(name))

    def update_send(self, parameters, loss, reuse_snapshot=False):
        """dpwa.py:104-123: publish (clock += 1, snapshot + {clock, loss}), then the
        Bernoulli fetch gate; under a DistGroup the fetch starts here on the side stream.

        reuse_snapshot (extension): the caller asserts `parameters` is unchanged since the
        last ``update_wait_average(..., write_through=True)``; the publish then writes only
        the header, the payload having been written by that average."""
        learner = self._learner
        if learner is None:
            learner = self._bind(parameters)
        elif learner.take_status():
            self._zero_division()
        p = learner._ptr(parameters)
        h, d, learner._keep = learner.loss_args(loss)
        s = self._raw_stream(learner.device.index)
        flags = self._flags | (_lib.FLAG_REUSE_SNAPSHOT if reuse_snapshot else 0)
        if self._eager:      # DistGroup: publish, stream-ordered barrier, gate + eager pull
            rc = self._f_publish(self._node, p, h, d, flags, s)
            if rc:
                self._fail("dpwa_node_publish", rc)
            self._group.after_publish(self)
            rc = self._f_gate(self._node, flags, s, self._out_ref)
            if not rc:
                self.fetching = bool(self._out.value)
                self._group.after_gate(self)
        else:
            rc = self._f_update_send(self._node, p, h, d, flags, s, self._out_ref)
        if rc:
            self._fail("dpwa_node_update_send", rc)
        learner.version += 1
        self.fetching = bool(self._out.value)
        if self._resident:      # the served snapshot: its version counter, checked at update_wait
            t = learner.resident_params()
            self._sent = (t, t._version)
        if not self._eager and getattr(self._group, "prefetch", False):
            self._group.after_update_send(self)

    def update_wait(self, loss):
        """dpwa.py:125-156: (None, 0) when not fetching or no peer delivered; otherwise the
        fetched snapshot and the device factor (the clock is updated on the device)."""
        learner = self._learner
        if learner is None:
            return None, 0
        if learner.take_status():
            self._zero_division()
        h, d, learner._keep = learner.loss_args(loss)
        rc = self._f_wait(self._node, h, d, self._flags, self._raw_stream(learner.device.index), self._out_ref)
        if rc:
            self._fail("dpwa_node_update_wait", rc)
        self.fetching = False
        return self._result()

    def update_wait_average(self, parameters, loss, write_through=False):
        """update_wait + the adapter's averaging (pytorch.py:60-68) as one fused kernel:
        the factor is evaluated inside the lerp.  Same results as update_wait() followed by
        average(); returns what update_wait returns.

        write_through (extension): the kernel also stores the averaged parameters into the
        next snapshot slot, so a following ``update_send(..., reuse_snapshot=True)`` moves
        no payload (4*n*s bytes for the round's averaging + publish instead of 5*n*s)."""
        learner = self._learner
        if learner is None:
            return None, 0
        if learner.take_status():
            self._zero_division()
        if self._sent is not None:
            self._check_window()
        p = learner._ptr(parameters)
        h, d, learner._keep = learner.loss_args(loss)
        flags = self._flags | (_lib.FLAG_WRITE_THROUGH if write_through else 0)
        rc = self._f_wait_avg(self._node, p, h, d, flags, self._raw_stream(learner.device.index), self._out_ref)
        if rc:
            self._fail("dpwa_node_update_wait_average", rc)
        self.fetching = False
        self._sent = None
        return self._result()

    # ---------------------------------------------------------------- extensions
    def make_resident(self, parameters):
        """Resident parameters (extension, dpwa_learner_set_resident in include/dpwa_hip.h): the
        parameters move into the learner's own snapshot slots, so a publish moves no bytes and the
        average reads them in the published slot and writes the next one -- 3*n*s bytes a round,
        the averaging's own.  Call before the first update_send; returns the tensor the
        parameters are in now (see ``parameters``).  From then on pass ``conn.parameters`` to
        update_send / update_wait_average, re-read it after every update_send and
        update_wait_average (it alternates between the two slots), and do not write it between
        update_send and update_wait_average: it is the served snapshot then.  So the loop is
        update_send, update_wait_average, step -- not the reference's update_send, step,
        update_wait (README.md:18-29, main.py:130-145), which needs the write-through or full
        form.  update_wait_average raises DpwaError when the tensor's version counter moved in
        that window (an in-place op on it or on a view of it; writes through ``.data`` are not
        counted)."""
        learner = self._learner if self._learner is not None else self._bind(parameters)
        stream = torch.cuda.current_stream(learner.device)
        learner._ptr(parameters)
        _lib.call("dpwa_node_set_resident", self._node, ctypes.c_void_p(parameters.data_ptr()),
                  ctypes.c_void_p(stream.cuda_stream))
        self._resident = True
        return learner.resident_params()

    @property
    def parameters(self):
        """The resident parameters' tensor now (None unless ``make_resident`` was called): a view
        of one of the learner's snapshot slots, valid until ``close``."""
        return self._learner.resident_params() if self._learner is not None else None

    @staticmethod
    def update_wait_average_many(conns, parameters, losses, write_through=False):
        """update_wait_average of several connections of this process (the learners of a
        LocalGroup): each fetch is resolved as the single calls would resolve it, and the
        averages of the learners that share a GPU run as ONE dispatch on that GPU's current
        stream instead of one per learner (same results; a kernel boundary and a launch
        ramp/drain fewer per extra learner).  Returns the list of what update_wait returns,
        per connection."""
        if not (len(conns) == len(parameters) == len(losses)):
            raise ValueError("update_wait_average_many: %d connections, %d buffers, %d losses"
                             % (len(conns), len(parameters), len(losses)))
        # the ctypes argument arrays of this set of connections, per device, reused across rounds
        # (the call is on the per-round path: its host cost must stay well under the dispatch it
        # replaces)
        key = tuple((c._node.value, c._learner.device.index) if c._learner is not None else None for c in conns)
        calls = _MANY_CALLS
        cache = calls.get(key)
        if cache is None:
            by_dev = {}
            for i, c in enumerate(conns):
                if c._learner is not None:
                    by_dev.setdefault(c._learner.device.index, []).append(i)
            cache = []
            for dev_index, bound in by_dev.items():     # one dispatch per device, node order kept
                k = len(bound)
                nodes = (ctypes.c_void_p * k)(*[conns[i]._node.value for i in bound])
                cache.append((bound, dev_index, nodes, (ctypes.c_void_p * k)(), (ctypes.c_double * k)(),
                              (ctypes.c_void_p * k)(), (ctypes.c_int * k)(), conns[bound[0]]._lib))
            if len(calls) > 64:
                calls.clear()
            calls[key] = cache
        for c in conns:         # resident learners: nothing wrote the served snapshots (before any call)
            if c._sent is not None:
                c._check_window()
        out = [(None, 0)] * len(conns)
        keep = []
        for bound, dev_index, nodes, flats, hs, ds, peers, lib in cache:
            flags = _lib.FLAG_WRITE_THROUGH if write_through else 0
            for j, i in enumerate(bound):
                c = conns[i]
                learner = c._learner
                if learner.take_status():
                    c._zero_division()
                flats[j] = learner._ptr(parameters[i])
                h, d, learner._keep = learner.loss_args(losses[i])
                keep.append(learner._keep)
                hs[j] = h
                ds[j] = d.value if d is not None else None
                flags |= c._flags
            rc = lib.dpwa_node_update_wait_average_many(nodes, flats, hs, ds, len(bound), flags,
                                                         torch._C._cuda_getCurrentRawStream(dev_index), peers)
            for i in bound:
                conns[i].fetching = False
                conns[i]._sent = None
            if rc:
                raise _lib.DpwaError("dpwa_node_update_wait_average_many", rc,
                                     lib.dpwa_last_error().decode(errors="replace"))
            for j, i in enumerate(bound):
                if peers[j] >= 0:
                    c = conns[i]
                    out[i] = (PeerSnapshot(c, peers[j], c._learner.version), DeviceFactor(c._learner))
        return out

    @property
    def clock(self):
        """The learner's clock (dpwa.py:59); reading it synchronises with the device."""
        if self._learner is None:
            return 0
        return self._learner.read_clock()

    def average(self, parameters, stream=None):
        """The lerp of pytorch.py:68 with the coefficients of the last update_wait."""
        learner = self._learner
        s = stream.cuda_stream if stream is not None else self._raw_stream(learner.device.index)
        rc = self._f_lerp(self._node, learner._ptr(parameters), s)
        if rc:
            self._fail("dpwa_node_lerp", rc)

    def synchronize(self):
        """Waits for the device and raises a deferred ZeroDivisionError, if any."""
        if self._learner is not None:
            torch.cuda.synchronize(self._learner.device)
        self._raise_pending()

    def inject_fault(self, peer_name, status):
        """Test/fault-injection hook: force a peer 'down' (refused), 'slow' (timeout),
        'dead' (unrecoverable) or 'no_state'; None clears it."""
        codes = {"down": _lib.PEER_DOWN, "slow": _lib.PEER_SLOW, "dead": _lib.PEER_DEAD,
                 "no_state": _lib.PEER_NO_STATE, "ready": _lib.PEER_READY}
        _lib.call("dpwa_node_set_fault", self._node, self._peer_by_name(peer_name),
                  -1 if status is None else codes[status])

    def state_dict(self):
        """Gossip state for a checkpoint (extension; the reference keeps none across a restart:
        dpwa.py:59 starts the clock at 0 and the process's `random` starts from its seed): the
        clock and the scheduler -- its generator, every peer's flow-control score and state, the
        peer order -- so a resumed job continues the same peer choices and clock bookkeeping.
        Plain data (ints, a float, strings): torch.save / json both take it."""
        return {"format": 1, "name": self.name, "peers": [p.name for p in self.peers],
                "clock": float(self.clock) if self._learner is not None else float(self._pending_clock or 0.0),
                "scheduler": self._sched.get_state()}

    def load_state_dict(self, state):
        """Restores a ``state_dict()`` taken from a connection with the same name and peers
        (before its first update_send, or between rounds)."""
        if state.get("format") != 1:
            raise ValueError("not a DpwaConnection state (format %r)" % state.get("format"))
        if state.get("name") != self.name or list(state.get("peers", [])) != [p.name for p in self.peers]:
            raise ValueError("state of node %r with peers %r does not fit node %r with peers %r"
                             % (state.get("name"), state.get("peers"), self.name, [p.name for p in self.peers]))
        self._sched.set_state(state["scheduler"])
        if self._learner is not None:
            self._learner.write_clock(float(state["clock"]))
        else:
            self._pending_clock = float(state["clock"])     # written once the learner exists (_bind)

    def flow_control_scores(self):
        return {p.name: self._sched.score(k) for k, p in enumerate(self.peers)}

    @property
    def last_fetch_attempts(self):
        return self._info()[3]

    @property
    def last_fetch_peer(self):
        k = self._info()[1]
        return None if k < 0 else self.peers[k].name

    def peer_rank(self, k):
        return self._peer_node_index[k]

    def close(self):
        """Shuts the node down; tensors from ``make_resident`` / ``parameters`` must not be used
        afterwards (their memory is the learner's)."""
        group = getattr(self, "_group", None)
        if group is not None:
            group.leave(self)
            self._group = None
        if getattr(self, "_learner", None) is not None:
            self._learner._h = None      # borrowed from the node
            self._learner = None
        node = getattr(self, "_node", None)
        if node is not None and node.value and _lib._lib is not None:
            _lib._lib.dpwa_node_destroy(node)
        self._node = None

    # ---------------------------------------------------------------- internals
    def _peer_by_name(self, name):
        k = self._peer_index.get(name)
        if k is None:
            raise KeyError(name)
        return k

    def _set_peer(self, k, kind, other):
        _lib.call("dpwa_node_set_peer", self._node, k, kind, other._node if other is not None else None)
        self._peer_wiring[k] = (kind, other.name if other is not None else None)

    def _info(self):
        fetching, peer, att = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        version = ctypes.c_uint64()
        _lib.call("dpwa_node_info", self._node, ctypes.byref(fetching), ctypes.byref(peer), ctypes.byref(version),
                  ctypes.byref(att))
        return bool(fetching.value), peer.value, version.value, att.value

    def _result(self):
        k = self._out.value
        if k < 0:
            return None, 0
        return PeerSnapshot(self, k, self._learner.version), DeviceFactor(self._learner)

    def _fail(self, name, rc):
        raise _lib.DpwaError(name, rc, self._lib.dpwa_last_error().decode(errors="replace"))

    def _bind(self, parameters):
        gpu = self.config.get_gpu(self.name)
        if gpu is not None and isinstance(parameters, torch.Tensor) and \
                (parameters.device.type != "cuda" or parameters.device.index != gpu):
            raise ValueError("node %r is placed on gpu %d by its config, but its parameters are on %s"
                             % (self.name, gpu, parameters.device))
        if not isinstance(parameters, torch.Tensor) or parameters.device.type != "cuda":
            raise TypeError("DpwaConnection.update_send expects the flat parameter buffer as a GPU tensor")
        if parameters.dtype not in DTYPES:
            # the reference's TYPE_CONVERSION lookup raises KeyError (pytorch.py:11-14, 22)
            raise KeyError("dpwa averages float32 or bfloat16 parameters, got %s" % parameters.dtype)
        _lib.call("dpwa_node_bind", self._node, parameters.device.index, parameters.numel(),
                  DTYPES[parameters.dtype])
        h = ctypes.c_void_p()
        _lib.call("dpwa_node_handles", self._node, ctypes.byref(h), None)
        self._learner = Learner(parameters.device, parameters.numel(), parameters.dtype, handle=h.value)
        if self._pending_clock is not None:           # load_state_dict before the first round
            self._learner.write_clock(self._pending_clock)
            self._pending_clock = None
        if self._pull.partition(":")[0] in RELAY_PULLS:
            if not hasattr(self._group, "relay_blocks"):
                raise ValueError("the relay pull needs a DistGroup (one learner per rank)")
            self._group.relay_blocks = 1     # allocate + exchange the relay buffers in on_bind
        self._group.on_bind(self)
        self.set_pull(self._pull)
        return self._learner

    def set_pull(self, mode):
        """Transport of copying fetches: 'copy' (hipMemcpyAsync on the side stream),
        'kernel[:blocks]' (pull kernel), 'relay[:blocks]' (DistGroup only, multi-link
        two-phase relay; the connection must have been created with a relay pull so the
        relay buffers exist) or 'relay-avg[:blocks]' (the same relay with its second phase
        fused into the average: the averaging kernel reads the peer's stripes where the first
        phase left them).  Every rank must switch between the same two rounds."""
        kind, _, blocks = mode.partition(":")
        if kind not in ("copy", "kernel") + RELAY_PULLS:
            raise ValueError("pull must be 'copy', 'kernel[:blocks]', 'relay[:blocks]' or 'relay-avg[:blocks]', "
                             "got %r" % mode)
        self._pull = mode
        learner = self._learner
        if learner is None:
            return
        torch.cuda.synchronize(learner.device)
        if kind in RELAY_PULLS:
            if not getattr(self._group, "relay_ready", False):
                raise ValueError("relay pull: create the connection with pull='relay' under a DistGroup")
            self._group.relay_blocks = int(blocks or 64)
            self._group.relay_fused = kind == "relay-avg"
            self._flags |= _lib.FLAG_PICK_ONLY
            return
        if getattr(self._group, "relay_blocks", 0):
            self._group.relay_blocks = 0
        self._flags &= ~_lib.FLAG_PICK_ONLY
        _lib.call("dpwa_learner_set_pull", learner.handle, _lib.PULL_KERNEL if kind == "kernel" else
                  _lib.PULL_COPY_ENGINE, int(blocks or 512))

    def _check_window(self):
        t, v = self._sent
        if t._version != v:
            raise _lib.DpwaError(
                "DpwaConnection.update_wait_average", _lib.ERR_STATE,
                "the resident parameters were modified between update_send and update_wait (version %d -> %d); "
                "they are the snapshot peers read in that window, so a resident loop runs update_send -> "
                "update_wait -> step.  The reference's order update_send -> step -> update_wait (README.md, "
                "main.py:130-145) needs the write-through or full form" % (v, t._version))

    def _zero_division(self):
        raise ZeroDivisionError("float division by zero (interpolation factor, dpwa.py:143-147)")

    def _raise_pending(self):
        if self._learner is not None and self._learner.take_status():
            self._zero_division()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
