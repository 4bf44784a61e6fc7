"""Gossip policy restated on the CPU -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, in plain Python over CPython's own MT19937 (``random.Random``, the
third-party algorithm the reference calls through the global ``random`` module):

* interpolation factors         dpwa/interpolation.py:13-15, 22-24, 31-33
* divergence scaling and clock  dpwa/dpwa.py:143-150
* Bernoulli fetch gate          dpwa/dpwa.py:101-102, 118-123
* peer choice + flow control    dpwa/conn.py:178-181, 224-272
* the fetch retry loop          dpwa/conn.py:274-317
"""
import random

FLOW_CONTROL_MIN_SCORE = 10      # conn.py:178
FLOW_CONTROL_MAX_SCORE = 1000    # conn.py:179
FLOW_CONTROL_INC_SCORE = 10      # conn.py:180
FLOW_CONTROL_DEC_SCORE = 100     # conn.py:181

METHODS = {"constant": 0, "clock": 1, "loss": 2}


def interpolation(method, value, clock, peer_clock, loss, peer_loss):
    """interpolation.py:13-15 (constant), 22-24 (clock), 31-33 (loss)."""
    if method == "constant":
        return value
    if method == "clock":
        return peer_clock / (clock + peer_clock)
    if method == "loss":
        return loss / (loss + peer_loss)
    raise KeyError(method)


def factor_and_clock(method, value, threshold, clock, peer_clock, loss, peer_loss):
    """dpwa.py:143-150: returns (factor, new_clock); ZeroDivisionError like the reference."""
    factor = interpolation(method, value, clock, peer_clock, loss, peer_loss)
    if loss < threshold:
        factor = factor * (loss / threshold)
    new_clock = factor * peer_clock + (1 - factor) * clock
    return factor, new_clock


class Peer:
    def __init__(self, name):
        self.name = name
        self.score = FLOW_CONTROL_MAX_SCORE     # conn.py:190
        self.connected = False                  # conn.py:193


class OracleLearner:
    """One learner's policy state: clock, fetching flag and its TxThread's peer table."""

    def __init__(self, name, peer_names, fetch_probability, method, value, threshold, seed):
        self.name = name
        self.rng = random.Random(seed)
        self.clock = 0                          # dpwa.py:59
        self.fetching = False
        self.fetch_probability = fetch_probability
        self.method, self.value, self.threshold = method, value, threshold
        self.peers = {n: Peer(n) for n in peer_names}   # insertion (YAML) order, conn.py:208-213

    # -- dpwa.py:104-123 --------------------------------------------------------
    def update_send(self, loss):
        self.clock += 1
        state = {"clock": self.clock, "loss": loss}
        self.fetching = self.rng.random() < self.fetch_probability
        return state

    # -- conn.py:224-262 --------------------------------------------------------
    def get_random_peer(self, connect_fn, attempts):
        scores = {k: v.score + self.rng.randint(FLOW_CONTROL_MIN_SCORE, FLOW_CONTROL_MAX_SCORE)
                  for k, v in self.peers.items()}
        if len(scores) == 0:
            return None
        max_score = max(scores.values())
        keys = [k for k, v in scores.items() if v == max_score]
        key = keys[self.rng.randint(0, len(keys) - 1)]
        peer = self.peers[key]
        if not peer.connected:
            out = connect_fn(key)
            attempts.append({"peer": key, "connect": out, "request": None})
            if out == "refused":
                peer.score = max(peer.score - FLOW_CONTROL_DEC_SCORE, FLOW_CONTROL_MIN_SCORE)
                return None
            if out == "error":
                del self.peers[key]
                return None
            peer.connected = True
        else:
            attempts.append({"peer": key, "connect": None, "request": None})
        return peer

    # -- conn.py:274-317 (one queue item) ----------------------------------------
    def fetch(self, connect_fn, request_fn, max_attempts=None, stop=None):
        """Returns (state, payload, attempts); state/payload None when no data.  stop (not the
        reference's): called after each request's outcome is applied; True ends the loop there
        without data -- the one case where the device path stops where TxThread would go on: the
        learner's own transport stuck (every rescue lane still pulling for DPWA_RESCUE_WAIT_MS,
        DESIGN §4)."""
        attempts = []
        while True:
            if max_attempts is not None and len(attempts) >= max_attempts:
                return None, None, attempts
            peer = self.get_random_peer(connect_fn, attempts)
            if peer is None:
                return None, None, attempts
            out, state, payload = request_fn(peer.name)
            attempts[-1]["request"] = out
            if out in ("payload", "empty"):
                peer.score = min(peer.score + FLOW_CONTROL_INC_SCORE, FLOW_CONTROL_MAX_SCORE)
                if out == "payload":
                    return state, payload, attempts
            elif out == "timeout":
                peer.score = max(peer.score - FLOW_CONTROL_DEC_SCORE, FLOW_CONTROL_MIN_SCORE)
                peer.connected = False
            else:  # unrecoverable request error: conn.py:311-313
                del self.peers[peer.name]
            if stop is not None and stop():
                return None, None, attempts

    # -- dpwa.py:125-156 --------------------------------------------------------
    def update_wait(self, loss, peer_state, have_payload):
        """Returns (averaged, factor); raises ZeroDivisionError like the reference."""
        if not self.fetching:
            return False, 0
        self.fetching = False
        if not have_payload:
            return False, 0
        factor, new_clock = factor_and_clock(self.method, self.value, self.threshold, self.clock,
                                             peer_state["clock"], loss, peer_state["loss"])
        self.clock = new_clock
        return True, factor

    # -- dpwa.py:95-96 -> conn.py:208-213 ----------------------------------------
    def add_peer(self, name):
        """A fresh WorkerConn under `name`: an existing key keeps its dict position, a
        removed one is inserted again at the end."""
        self.peers[name] = Peer(name)

    def scores(self, names):
        return [self.peers[n].score if n in self.peers else None for n in names]
