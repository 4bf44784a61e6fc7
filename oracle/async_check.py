"""Checker for free-running (gossip-board) rounds -- TEST INFRASTRUCTURE ONLY (see
oracle/__init__.py).  Used by tests/test_gpu_async.py and by bench.py's parity leg, after
the timed region, never as the thing measured.

In a free-running round the version of a peer that gets averaged depends on timing, so there
is no fixed trajectory to replay.  Instead every rank publishes parameters that are a known
function of (rank, round) -- ``async_base`` -- and losses ``async_loss``; then a round that
read version v of peer q must equal the oracle lerp (pytorch.py:68) of this round's base
with q's base of round v-1 under the factor of dpwa.py:143-147, and the clocks must follow
dpwa.py:112 and 150-155 through exactly the versions that were read.  A torn or overwritten
snapshot, a version handed out before its bytes landed or a stale clock cannot pass.
"""
import hashlib

import numpy as np

from .lerp import bits_equal, f32_to_bf16, lerp_f32
from .policy import factor_and_clock


def async_base(rank, r, n):
    """The parameters rank `rank` publishes at its round r (publish number r + 1)."""
    return (np.arange(n, dtype=np.float32) * np.float32(1e-3) + np.float32(rank * 1000 + r)).astype(np.float32)


def async_base_bf16(rank, r, n):
    """async_base rounded to bf16 (raw bits), for the bf16 runs."""
    return f32_to_bf16(async_base(rank, r, n))


def async_loss(rank, r, wait=False):
    """The loss rank `rank` passes at its round r (update_send, or update_wait when `wait`):
    decaying, so a divergence threshold is crossed mid-run."""
    x = 2.0 * float(np.exp(-r / 8.0)) + 0.1 * rank + 0.05
    return 0.9 * x if wait else x


def digest(a):
    """sha1 of an array's bytes (bit-exact comparison without moving the array)."""
    return hashlib.sha1(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


class AsyncRuns:
    """Recomputes the clocks and factors of a set of free-running runs.

    peers[g][r]    name of the peer rank g averaged with at its round r ("" = none)
    versions[g][r] the version (1-based publish number) of that peer it read
    names          node names, index = rank
    Only ranks present in `peers` are known; a rank that left early is absent."""

    def __init__(self, names, peers, versions, interp="constant", value=0.5, thr=0.0, published=None,
                 base=async_base, lerp=lerp_f32):
        """published(q, v, n): the parameters rank q published as version v (1-based).  Default:
        base(q, v - 1, n), the runs whose every round publishes its known base.  Runs with
        write-through snapshots publish what their last round averaged; pass those.  base and
        lerp give the dtype: async_base / lerp_f32, or their bf16 forms (raw bits)."""
        self.base, self.lerp = base, lerp
        self.published = published or (lambda q, v, n: self.base(q, v - 1, n))
        self.names = list(names)
        self.peers = {g: [str(p) for p in v] for g, v in peers.items()}
        self.versions = {g: [int(x) for x in v] for g, v in versions.items()}
        self.interp, self.value, self.thr = interp, value, thr
        self._after = {}

    def complete(self):
        return all(g in self.peers for g in range(len(self.names)))

    def read(self, g, r):
        """(peer rank, version) read by rank g at round r, or None."""
        p = self.peers[g][r]
        if p == "":
            return None
        return self.names.index(p), self.versions[g][r]

    def policy(self, g, r):
        """dpwa.py:143-155 for rank g's round r against what it read: (factor, new clock)."""
        q, v = self.read(g, r)
        return factor_and_clock(self.interp, self.value, self.thr, self.clock_published(g, r),
                                self.clock_published(q, v - 1), async_loss(g, r, True), async_loss(q, v - 1))

    def clock_published(self, g, r):
        """The clock rank g published at its round r (dpwa.py:112: clock += 1)."""
        return (self.clock_after(g, r - 1) if r > 0 else 0.0) + 1.0

    def clock_after(self, g, r):
        """Rank g's clock after its round r's update_wait (dpwa.py:155; unchanged with no data)."""
        key = (g, r)
        if key not in self._after:
            if self.read(g, r) is None:
                self._after[key] = self.clock_published(g, r)
            else:
                self._after[key] = self.policy(g, r)[1]
        return self._after[key]

    def expected_params(self, g, r, n):
        """What rank g's parameters must be after round r."""
        mine = self.base(g, r, n)
        got = self.read(g, r)
        if got is None:
            return mine
        q, v = got
        if self.complete():
            factor = self.policy(g, r)[0]
        else:           # a departed rank's clocks are unknown: constant interpolation only
            if not (self.interp == "constant" and self.thr == 0.0):
                raise ValueError("incomplete runs can only be checked under constant interpolation")
            factor = self.value
        return self.lerp(mine, self.published(q, v, n), factor)

    def check_rank(self, g, params, clocks, n):
        """Checks rank g's recorded params (T x n) and clocks (T) round by round; returns a list
        of failure strings (empty = every round matched bit for bit)."""
        bad = []
        last = {}
        for r in range(len(self.peers[g])):
            got = self.read(g, r)
            if got is not None:
                q, v = got
                if v < 1:
                    bad.append("round %d: version %d" % (r, v))
                if v < last.get(q, 0):
                    bad.append("round %d: versions of %s went backwards" % (r, self.names[q]))
                last[q] = v
            want = self.expected_params(g, r, n)
            if not bits_equal(np.asarray(params[r]), want):
                bad.append("round %d: parameters differ from the oracle (peer %s)" % (r, self.peers[g][r] or "-"))
            if self.complete() and float(clocks[r]) != self.clock_after(g, r):
                bad.append("round %d: clock %r != %r" % (r, float(clocks[r]), self.clock_after(g, r)))
        return bad

    # -- distributed form: no rank needs another rank's parameters ------------------------
    def served(self, q, published_by_q, n):
        """Digests of what every average that read a version published by rank q must equal:
        {(reader g, round r): digest}.  Run on rank q, which holds its own published
        snapshots (published_by_q(v) -> array), e.g. write-through runs that publish what
        their last round averaged."""
        out = {}
        for g in self.peers:
            for r in range(len(self.peers[g])):
                got = self.read(g, r)
                if got is None or got[0] != q:
                    continue
                factor = self.policy(g, r)[0] if self.complete() else self.value
                out[(g, r)] = digest(self.lerp(self.base(g, r, n), published_by_q(got[1]), factor))
        return out

    def check_rank_digests(self, g, params, clocks, n, expected):
        """check_rank with the averages compared against `expected` (the union of every
        publisher's served()); rounds with no data must leave async_base(g, r)."""
        bad = []
        last = {}
        for r in range(len(self.peers[g])):
            got = self.read(g, r)
            if got is None:
                if digest(params[r]) != digest(self.base(g, r, n)):
                    bad.append("round %d: parameters changed without an average" % r)
            else:
                q, v = got
                if v < 1 or v < last.get(q, 0):
                    bad.append("round %d: version %d of %s out of order" % (r, v, self.names[q]))
                last[q] = v
                if digest(params[r]) != expected.get((g, r)):
                    bad.append("round %d: average differs from %s's published version %d" % (r, self.names[q], v))
            if self.complete() and float(clocks[r]) != self.clock_after(g, r):
                bad.append("round %d: clock %r != %r" % (r, float(clocks[r]), self.clock_after(g, r)))
        return bad
