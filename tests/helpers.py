"""Shared helpers for the test-suite (fixture loading, outcome replay)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def num(x):
    if isinstance(x, str):
        return float(x)
    return x


def hexf(s):
    return float.fromhex(s)


class AttemptReplay:
    """Feeds recorded (connect, request) outcomes back, attempt by attempt, and
    checks that the replayed scheduler picks the same peer each time."""

    def __init__(self, attempts, reply=None):
        self.attempts = attempts
        self.i = 0
        self.reply = reply or (lambda peer: ({"clock": 1 + int(peer[1:]), "loss": 0.5}, b"payload"))
        self.picked = []

    def connect(self, peer):
        a = self.attempts[self.i]
        assert a["peer"] == peer, (self.i, a, peer)
        assert a["connect"] is not None
        self.picked.append(peer)
        out = a["connect"]
        if out != "ok":
            self.i += 1
        return out

    def request(self, peer):
        a = self.attempts[self.i]
        assert a["peer"] == peer, (self.i, a, peer)
        if a["connect"] is None:
            self.picked.append(peer)
        self.i += 1
        out = a["request"]
        if out == "payload":
            st, pl = self.reply(peer)
            return out, st, pl
        return out, None, None

    def done(self):
        return self.i == len(self.attempts)


# ---- measured holds for the fetch-timeout tests (test_gpu_timeout.py, dist_worker.py) ----------
TIMEOUT_MS = 100                 # the YAML's timeout_ms in the timed-out rounds
HOST_WAIT_S = 0.3                # the host waits this long after update_send: 3 x timeout_ms
HOLD_S = 0.9                     # a held pull's spin: 3 x the host wait
assert HOST_WAIT_S >= 3 * TIMEOUT_MS / 1e3 and HOLD_S >= 3 * HOST_WAIT_S


def sleep_rate():
    """torch.cuda._sleep cycles per second on this box: two spins of different length timed by
    events, the rate from their difference (launch overhead cancels)."""
    import torch

    def timed(cycles):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda._sleep(cycles)
        b.record()
        b.synchronize()
        return a.elapsed_time(b) * 1e-3
    timed(10_000_000)
    short, long_ = timed(20_000_000), timed(220_000_000)
    return 200_000_000 / max(long_ - short, 1e-6)


class Hold:
    """A spin of `seconds` (from the measured rate) on `stream`, timed by events, so the test can
    state afterwards how long the pull behind it was really held."""
    rate = None

    def __init__(self, stream, seconds=HOLD_S):
        import torch
        if Hold.rate is None:
            Hold.rate = sleep_rate()
        self.seconds = seconds
        self.a, self.b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            self.a.record()
            torch.cuda._sleep(int(seconds * Hold.rate))
            self.b.record()

    def check(self, waited_s):
        """After the round: the hold outlasted the host's wait past the deadline by >= 2x."""
        held = self.a.elapsed_time(self.b) * 1e-3
        assert held >= 2 * waited_s, ("the hold lasted %.0f ms, under 2 x the host's %.0f ms wait past the %d ms "
                                      "deadline (spin rate %.3g cycles/s): the held pull may have landed before it "
                                      "was judged" % (1e3 * held, 1e3 * waited_s, TIMEOUT_MS, Hold.rate))
        return held


GUARD_SAMPLES = 4096


def guard_words(n16, gen, samples=GUARD_SAMPLES):
    """The 16-B words the reuse / window guard compares at publish generation `gen` (a host
    restatement of kernels.hip guard_offset): the payload is cut into min(n16, 4096) chunks,
    chunk k = words [b(k), b(k+1)) with b(k) = k(n16-1)/(s-1) (the last chunk is the last word
    alone), and chunk k is sampled at word b(k) + gen mod (its length); the first word is compared
    at every generation too.  Every word is covered in any W consecutive generations."""
    s = min(n16, samples)
    if s <= 1:
        return {0, max(0, n16 - 1)}

    def b(k):
        return k * (n16 - 1) // (s - 1)
    out = {b(k) + gen % (b(k + 1) - b(k)) for k in range(s - 1)}
    return out | {0, n16 - 1}


def guard_chunk(n16, word, samples=GUARD_SAMPLES):
    """The chunk (index) a word belongs to, and its word range."""
    s = min(n16, samples)
    if s <= 1 or word >= n16 - 1:
        return max(0, s - 1), (max(0, n16 - 1), n16)
    k = word * (s - 1) // (n16 - 1)
    while k * (n16 - 1) // (s - 1) > word:
        k -= 1
    while (k + 1) * (n16 - 1) // (s - 1) <= word:
        k += 1
    return k, (k * (n16 - 1) // (s - 1), (k + 1) * (n16 - 1) // (s - 1))


def guard_period(n16, samples=GUARD_SAMPLES):
    """W: the longest chunk, so every word is sampled within W consecutive generations."""
    s = min(n16, samples)
    if s <= 1:
        return 1
    return max((k + 1) * (n16 - 1) // (s - 1) - k * (n16 - 1) // (s - 1) for k in range(s - 1))
