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
import logging

import torch
import yaml

from . import _lib
from .group import default_group
from .interpolation import INTERPOLATION_METHODS
from .learner import Learner
from .sched import Scheduler

LOGGER = logging.getLogger(__name__)

MAX_FETCH_ATTEMPTS = 100000   # the reference loops forever when every peer keeps timing out


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
    def get_seed(self, name):
        """Per-node `seed:` key, else a top-level `- seed:` entry, else None (OS entropy,
        as the reference, which never seeds `random`)."""
        for node in self.get_nodes():
            if node.get('name') == name and 'seed' in node:
                return node['seed']
        return self.config.get('seed')


class PeerSnapshot:
    """What update_wait returns in place of the reference's pickled payload bytes: the
    fetched snapshot, resident on the learner's GPU."""

    def __init__(self, conn, peer_index, version):
        self.peer = conn.peers[peer_index].name
        self.version = version
        self.numel = conn._learner.numel
        self.dtype = conn._learner.dtype

    def __repr__(self):
        return "PeerSnapshot(peer=%r, version=%d, numel=%d, dtype=%s)" % (self.peer, self.version, self.numel,
                                                                          self.dtype)


class DeviceFactor:
    """The interpolation factor, computed on the device.  ``float(f)`` synchronises."""

    def __init__(self, learner):
        self._learner = learner

    def __float__(self):
        return float(self._learner.read_coef().factor)

    def coefficients(self):
        c = self._learner.read_coef()
        return {"factor": c.factor, "new_clock": c.new_clock, "a": c.a, "b": c.b, "status": c.status}

    def __repr__(self):
        return "DeviceFactor(%r)" % float(self)


class DpwaConnection:
    def __init__(self, name, config_file, seed=None, group=None):
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

        # Interpolation method (dpwa.py:75-80)
        interpolation_method, interpolation_config = self.config.get_interpolation()
        LOGGER.debug("Using %s interpolation method", interpolation_method)
        if interpolation_config == 0:
            interpolation_config = {}
        self.interpolation = INTERPOLATION_METHODS[interpolation_method](**interpolation_config)
        self.divergence_threshold = self.config.get_divergence_threshold()
        self.timeout_ms = self.config.get_timeoutms()

        # TxThread's replacement: the scheduler (conn.py:197-334)
        if seed is None:
            seed = self.config.get_seed(name)
        self._sched = Scheduler(len(self.peers), seed, self.fetch_probability)
        self._status_buf = self._sched.status_buffer()
        self._faults = {}
        self._attached = {}
        self._learner = None
        self._fetch_peer = -1
        self._fetch_started = False
        self.last_fetch_attempts = 0
        self._group = group if group is not None else default_group(config_file, self.nodes, name)
        self._group.join(self)

    # ---------------------------------------------------------------- reference API
    def add_peer(self, name, host, port):
        raise NotImplementedError("peers come from the YAML node list (dpwa.py:88-89); "
                                  "re-adding a removed peer is not supported")

    def remove_peer(self, name):
        """dpwa.py:98-99 -> TxThread.remove_peer (conn.py:215-222): permanent."""
        k = self._peer_by_name(name)
        _lib.call("dpwa_sched_remove", self._sched._h, k)

    def update_send(self, parameters, loss):
        """dpwa.py:104-123: publish (clock += 1, snapshot + {clock, loss}), then the
        Bernoulli fetch gate; under a DistGroup the fetch starts here on the side stream."""
        learner = self._learner
        if learner is None:
            learner = self._bind(parameters)
        elif learner.take_status():
            self._zero_division()
        stream = torch.cuda.current_stream(learner.device)
        learner.publish(parameters, loss, stream)
        self._group.after_publish(self, stream)
        self._fetch_started = False
        self._fetch_peer = -1
        if self._sched.bernoulli():
            LOGGER.debug("update_send(): starting fetch parameters request")
            self.fetching = True
            if self._group.eager_fetch:
                self._start_fetch(stream)
        else:
            self.fetching = False

    def update_wait(self, loss):
        """dpwa.py:125-156: (None, 0) when not fetching or no peer delivered; otherwise the
        fetched snapshot and the device factor (the clock is updated on the device)."""
        stream = self._finish_fetch()
        if stream is None:
            return None, 0
        self._learner.factor(loss, stream)
        return PeerSnapshot(self, self._fetch_peer, self._fetch_version), DeviceFactor(self._learner)

    def update_wait_average(self, parameters, loss):
        """update_wait + the adapter's averaging (pytorch.py:60-68) as one fused kernel:
        the factor is evaluated inside the lerp.  Same results as update_wait() followed by
        average(); returns what update_wait returns."""
        stream = self._finish_fetch()
        if stream is None:
            return None, 0
        self._learner.average(parameters, loss, stream)
        return PeerSnapshot(self, self._fetch_peer, self._fetch_version), DeviceFactor(self._learner)

    # ---------------------------------------------------------------- extensions
    @property
    def clock(self):
        """The learner's clock (dpwa.py:59); reading it synchronises with the device."""
        if self._learner is None:
            return 0
        return self._learner.read_clock()

    def average(self, parameters, stream=None):
        """The lerp of pytorch.py:68 with the coefficients of the last update_wait."""
        self._learner.lerp(parameters, stream if stream is not None else torch.cuda.current_stream(self._learner.device))

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
        self._peer_by_name(peer_name)
        if status is None:
            self._faults.pop(peer_name, None)
        else:
            self._faults[peer_name] = codes[status]

    def flow_control_scores(self):
        return {p.name: self._sched.score(k) for k, p in enumerate(self.peers)}

    def peer_rank(self, k):
        return self._peer_node_index[k]

    def close(self):
        self._group.leave(self)
        if self._learner is not None:
            self._learner.close()
            self._learner = None

    # ---------------------------------------------------------------- internals
    def _peer_by_name(self, name):
        for k, p in enumerate(self.peers):
            if p.name == name:
                return k
        raise KeyError(name)

    def _bind(self, parameters):
        if not isinstance(parameters, torch.Tensor) or parameters.device.type != "cuda":
            raise TypeError("DpwaConnection.update_send expects the flat parameter buffer as a GPU tensor")
        cfg = self.interpolation.device_config(self.divergence_threshold)
        self._learner = Learner(parameters.device, parameters.numel(), parameters.dtype, cfg)
        self._group.on_bind(self)
        return self._learner

    def _finish_fetch(self):
        """dpwa.py:130-137: returns the stream to average on, or None for "no data"."""
        learner = self._learner
        if learner is not None and learner.take_status():
            self._zero_division()
        if not self.fetching:
            return None
        self.fetching = False
        stream = torch.cuda.current_stream(learner.device)
        if not self._fetch_started:
            self._start_fetch(stream)
        if self._fetch_peer < 0:
            return None
        return stream

    def _start_fetch(self, stream):
        """TxThread.run for one queue item (conn.py:277-315) + the pull itself."""
        self._fetch_started = True
        status = self._status_buf
        group = self._group
        for k, p in enumerate(self.peers):
            st = self._faults.get(p.name) if self._faults else None
            status[k] = group.peer_status(self, p.name) if st is None else st
        k, attempts = self._sched.fetch_into(status, MAX_FETCH_ATTEMPTS)
        self.last_fetch_attempts = attempts
        self._fetch_peer = k
        if k < 0:
            return
        version, zero_copy = group.prepare_fetch(self, k)
        self._fetch_version = version
        self._learner.fetch(k, version, zero_copy, stream)

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
