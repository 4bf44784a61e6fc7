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
