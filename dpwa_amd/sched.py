"""Host-side gossip scheduler: the reference TxThread's peer choice and flow control
(dpwa/conn.py:178-317) and the Bernoulli gate (dpwa/dpwa.py:101-102), implemented in C++
(dpwa_amd/csrc/sched.cpp) over a CPython-exact MT19937.

``Scheduler(n_peers, seed, p)`` draws exactly what a reference process that called
``random.seed(seed)`` draws, in the same order: ``random()`` for the gate, then per pick
one ``randint(10, 1000)`` per live peer plus the tie-break ``randint(0, k-1)``.
"""
import ctypes

from . import _lib

# conn.py:178-181 (the native scheduler's bounds, dpwa_amd/csrc/sched.cpp)
FLOW_CONTROL_MIN_SCORE = 10
FLOW_CONTROL_MAX_SCORE = 1000
FLOW_CONTROL_INC_SCORE = 10
FLOW_CONTROL_DEC_SCORE = 100

OUTCOMES = {
    "connect_ok": _lib.CONNECT_OK, "refused": _lib.CONNECT_REFUSED, "connect_error": _lib.CONNECT_ERROR,
    "payload": _lib.REPLY_PAYLOAD, "empty": _lib.REPLY_EMPTY, "timeout": _lib.REPLY_TIMEOUT,
    "error": _lib.REPLY_ERROR,
}


def seed_key(seed):
    """32-bit little-endian words of abs(seed), as CPython's random.seed(int) splits it."""
    n = abs(int(seed))
    words = []
    while n:
        words.append(n & 0xFFFFFFFF)
        n >>= 32
    return words   # [] == seed 0 (key [0])


class Scheduler:
    def __init__(self, n_peers, seed=None, fetch_probability=1.0, handle=None):
        self._owned = handle is None
        self._h = ctypes.c_void_p() if handle is None else ctypes.c_void_p(handle)
        if handle is not None:
            pass                  # the node's scheduler, borrowed (dpwa_node_handles)
        elif seed is None:
            _lib.call("dpwa_sched_create", ctypes.byref(self._h), n_peers, None, -1, float(fetch_probability))
        else:
            key = seed_key(seed)
            arr = (ctypes.c_uint32 * max(1, len(key)))(*key)
            _lib.call("dpwa_sched_create", ctypes.byref(self._h), n_peers, arr, len(key), float(fetch_probability))
        self.n_peers = n_peers
        self._f_fetch = _lib.load().dpwa_sched_fetch
        self._peer_out, self._att_out = ctypes.c_int(), ctypes.c_int()
        self._peer_ref, self._att_ref = ctypes.byref(self._peer_out), ctypes.byref(self._att_out)

    def __del__(self):
        h = getattr(self, "_h", None)
        if getattr(self, "_owned", False) and h and h.value and _lib._lib is not None:
            _lib._lib.dpwa_sched_destroy(h)
            self._h = None

    def bernoulli(self):
        out = ctypes.c_int()
        _lib.call("dpwa_sched_bernoulli", self._h, ctypes.byref(out))
        return bool(out.value)

    def pick(self):
        """Returns (peer index or -1, connected)."""
        peer, conn = ctypes.c_int(), ctypes.c_int()
        _lib.call("dpwa_sched_pick", self._h, ctypes.byref(peer), ctypes.byref(conn))
        return peer.value, bool(conn.value)

    def report(self, peer, outcome):
        """Returns (round_done, got_data)."""
        if isinstance(outcome, str):
            outcome = OUTCOMES[outcome]
        done, data = ctypes.c_int(), ctypes.c_int()
        _lib.call("dpwa_sched_report", self._h, peer, outcome, ctypes.byref(done), ctypes.byref(data))
        return bool(done.value), bool(data.value)

    def fetch(self, peer_status, max_attempts=1000):
        """Whole TxThread fetch loop against a static per-peer status list; returns (peer, attempts)."""
        arr = (ctypes.c_int32 * max(1, len(peer_status)))(*peer_status)
        peer, att = ctypes.c_int(), ctypes.c_int()
        _lib.call("dpwa_sched_fetch", self._h, arr, max_attempts, ctypes.byref(peer), ctypes.byref(att))
        return peer.value, att.value

    def status_buffer(self):
        """A reusable per-peer status array for fetch_into()."""
        return (ctypes.c_int32 * max(1, self.n_peers))()

    def fetch_into(self, status_buf, max_attempts=1000):
        """fetch() on a buffer from status_buffer() (no per-call allocation)."""
        peer, att = self._peer_out, self._att_out
        rc = self._f_fetch(self._h, status_buf, max_attempts, self._peer_ref, self._att_ref)
        if rc:
            raise _lib.DpwaError("dpwa_sched_fetch", rc, _lib.load().dpwa_last_error().decode(errors="replace"))
        return peer.value, att.value

    def add(self, peer):
        """TxThread.add_peer (conn.py:208-213): fresh record, score 1000, not connected."""
        _lib.call("dpwa_sched_add", self._h, peer)

    def remove(self, peer):
        _lib.call("dpwa_sched_remove", self._h, peer)

    def score(self, peer):
        out = ctypes.c_int()
        _lib.call("dpwa_sched_score", self._h, peer, ctypes.byref(out))
        return None if out.value < 0 else out.value

    def scores(self):
        return [self.score(k) for k in range(self.n_peers)]

    def n_live(self):
        out = ctypes.c_int()
        _lib.call("dpwa_sched_n_live", self._h, ctypes.byref(out))
        return out.value

    def get_state(self):
        """The scheduler's whole state as a list of 32-bit words (include/dpwa_hip.h
        dpwa_sched_get_state): words 2..626 are CPython's random.getstate()[1]."""
        n = ctypes.c_int()
        _lib.call("dpwa_sched_get_state", self._h, None, 0, ctypes.byref(n))
        buf = (ctypes.c_uint32 * n.value)()
        _lib.call("dpwa_sched_get_state", self._h, buf, n.value, ctypes.byref(n))
        return list(buf)

    def set_state(self, words):
        buf = (ctypes.c_uint32 * len(words))(*[int(w) for w in words])
        _lib.call("dpwa_sched_set_state", self._h, buf, len(words))

    def random(self):
        out = ctypes.c_double()
        _lib.call("dpwa_sched_random", self._h, ctypes.byref(out))
        return out.value

    def randint(self, a, b):
        out = ctypes.c_int64()
        _lib.call("dpwa_sched_randint", self._h, a, b, ctypes.byref(out))
        return out.value
