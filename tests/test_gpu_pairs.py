"""Shared reads in the resident batched dispatch (kernels.hip launch_average_batch): co-resident
resident learners read each other's published slots -- two that average with each other both read
both slots, and a slot is read by its owner and by every learner that picked it.  A mutual pair
(two entries, each the other's peer: the N=1 loop) runs as k_lerp_pair, and any other group of
equal-size entries whose reads overlap as k_lerp_group (up to eight distinct buffers: the entries'
parameters and the peers outside the dispatch), one workgroup per span loading every buffer once
and storing all the averages; sharing batches beyond eight buffers run k_lerp_batch's
XCD-grouped span order (every entry's span s on XCD s % 8, one after the other, so
the later reads of a span hit that XCD's L2).  Either way every entry must still be exactly the
single-learner fused average (factor, clock, lerp into the next slot, ragged tail, ZeroDivision
no-op) against the CPU oracle, whatever the mix of sharing and non-sharing entries in the
dispatch, and the published slots must stay untouched."""
import ctypes

import numpy as np
import pytest
import torch

from dpwa_amd import DpwaConnection, _lib
from dpwa_amd.group import LocalGroup
from oracle import gossip as ogossip
from oracle import lerp as olerp
from oracle import policy as opolicy
from tests.test_gpu_kernels import average_slot, from_u16, stream, to_u16

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
OFF = _lib.SLOT_PAYLOAD_OFFSET


class Learner:
    """A resident learner as the batch sees it: its published slot (header + parameters), its next
    slot, its clock pair and coefficient block."""

    def __init__(self, n, dtype, rng, clock, loss):
        self.n, self.dtype = n, dtype
        p32 = rng.standard_normal(n).astype(np.float32)
        self.host = p32 if dtype == "f32" else olerp.f32_to_bf16(p32)
        t = torch.from_numpy(p32).to(DEV) if dtype == "f32" else from_u16(self.host)
        self.clock_val, self.loss = clock, loss
        self.slot = average_slot(t, clock, loss)           # the published snapshot = the parameters
        self.esize = 4 if dtype == "f32" else 2
        self.next = torch.full((OFF + n * self.esize,), 0x7f, dtype=torch.uint8, device=DEV)
        self.clock = torch.tensor([clock, -1.0], dtype=torch.float64, device=DEV)
        self.coef = torch.zeros(32, dtype=torch.uint8, device=DEV)

    def payload(self, slot):
        raw = slot[OFF:].cpu().numpy()
        return raw.view(np.float32) if self.dtype == "f32" else raw.view(np.uint16)


def _desc(me, peer, loss):
    return _lib.AverageDesc(me.slot.data_ptr() + OFF, peer.slot.data_ptr(), me.n, me.clock.data_ptr(), loss,
                            me.coef.data_ptr(), me.next.data_ptr() + OFF)


def _expect(me, peer, method, loss):
    res = opolicy.factor_and_clock(method, None, 0.0, me.clock_val, peer.clock_val, loss, peer.loss) \
        if not (method == "loss" and loss + peer.loss == 0.0) else None
    exp = me.host.copy()
    if res is not None:
        (olerp.c_lerp_f32_ if me.dtype == "f32" else olerp.c_lerp_bf16_)(exp, np.ascontiguousarray(peer.host[:me.n]),
                                                                         res[0])
    return exp, res


def _run(learners, picks, dtype, method="clock", losses=None, env_off=False):
    """picks: [(me, peer)] in descriptor order; returns per entry (got, expected, res)."""
    losses = losses or [0.5 + 0.1 * i for i in range(len(picks))]
    d = (_lib.AverageDesc * len(picks))()
    for j, ((a, b), loss) in enumerate(zip(picks, losses)):
        d[j] = _desc(learners[a], learners[b], loss)
    before = [lr.slot.clone() for lr in learners]
    cfg = _lib.Interp(opolicy.METHODS[method], 0, 0.0, 0.0)
    _lib.call("dpwa_average_many_resident", _lib.F32 if dtype == "f32" else _lib.BF16, d, len(picks),
              ctypes.byref(cfg), stream(), None, None)
    torch.cuda.synchronize()
    for lr, b in zip(learners, before):
        assert torch.equal(lr.slot, b)                   # the published snapshots are only read
    out = []
    for (a, b), loss in zip(picks, losses):
        me = learners[a]
        exp, res = _expect(me, learners[b], method, loss)
        out.append((me.payload(me.next), exp, res, me))
    return out


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("n", [1, 7, 64 * 4, 8 * 64 * 4 - 1, 8 * 64 * 4, 8 * 64 * 4 + 1, 4099, 65536 + 13,
                               (1 << 20) + 5])
def test_mutual_pair_vs_oracle(dtype, n):
    """One mutual pair at sizes around the 8-span group of the XCD pairing (a partial last group,
    an exact multiple, one element over) and ragged tails: both averages bit-exact with the C
    oracle, both clocks and coefficient blocks written."""
    rng = np.random.default_rng(n)
    ls = [Learner(n, dtype, rng, 1.0, 0.5), Learner(n, dtype, rng, 4.0, 0.75)]
    for got, exp, res, me in _run(ls, [(0, 1), (1, 0)], dtype):
        assert olerp.bits_equal(got, exp), n
        c = _lib.Coef.from_buffer_copy(me.coef.cpu().numpy().tobytes())
        assert c.status == 0 and c.factor == res[0]
        assert me.clock[1].item() == res[1]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("mixed", [False, True])
def test_shared_reads_in_one_dispatch(dtype, mixed):
    """Seven learners' averages in one dispatch, descriptors in a scrambled order: two mutual
    pairs, a slot read by three learners, entries whose peer reads someone else; all sizes equal
    (a closed group of eight: k_lerp_group) or one entry smaller (the batch's span orders)."""
    rng = np.random.default_rng(3)
    n = 8 * 64 * 4 * 3 + 4099
    sizes = [n] * 8
    if mixed:
        sizes[5] = 123
    ls = [Learner(m, dtype, rng, 1.0 + i, 0.25 + 0.1 * i) for i, m in enumerate(sizes)]
    picks = [(2, 6), (0, 3), (6, 2), (4, 0), (3, 0), (7, 2), (1, 4)] + ([(5, 1)] if mixed else [(5, 0)])
    for got, exp, _, me in _run(ls, picks, dtype):
        assert olerp.bits_equal(got, exp)


CLOSED = {
    "3-cycle": [(0, 1), (1, 2), (2, 0)],
    "3-star": [(0, 1), (1, 0), (2, 0)],
    "4-two-pairs": [(3, 2), (0, 1), (2, 3), (1, 0)],
    "4-shared": [(0, 1), (1, 0), (2, 1), (3, 1)],
    "5": [(0, 4), (1, 0), (2, 0), (3, 2), (4, 3)],
    "6": [(5, 0), (0, 5), (1, 2), (2, 1), (3, 4), (4, 3)],
    "7": [(i, (i + 3) % 7) for i in range(7)],
}


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("name", sorted(CLOSED))
@pytest.mark.parametrize("n", [5, 8 * 64 * 4 * 3 + 4099])
def test_closed_groups_vs_oracle(dtype, name, n):
    """Co-resident resident learners that all picked learners of the same dispatch (a closed group:
    cycles, stars, two mutual pairs, one slot read by three) run as k_lerp_group, one workgroup per
    span loading every slot once: each entry bit-exact with the C oracle, ragged tails included."""
    picks = CLOSED[name]
    rng = np.random.default_rng(len(name) + n)
    ls = [Learner(n, dtype, rng, 1.0 + 0.5 * i, 0.2 + 0.1 * i) for i in range(len(picks))]
    for got, exp, _, me in _run(ls, picks, dtype):
        assert olerp.bits_equal(got, exp)


def test_closed_group_with_zero_division_entries():
    """Loss interpolation in a closed group of four where two entries have loss + peer loss == 0:
    those copy their parameters into their next slots and keep their clocks; the others average."""
    rng = np.random.default_rng(23)
    n = 70_003
    ls = [Learner(n, "f32", rng, 2.0 + i, 0.0 if i in (0, 1) else 0.3 * i) for i in range(4)]
    picks = [(0, 1), (1, 0), (2, 3), (3, 2)]
    out = _run(ls, picks, "f32", method="loss", losses=[0.0, 0.0, 0.4, 0.7])
    for k, (got, exp, res, me) in enumerate(out):
        c = _lib.Coef.from_buffer_copy(me.coef.cpu().numpy().tobytes())
        if k < 2:
            assert res is None and olerp.bits_equal(got, me.host) and c.status == _lib.STATUS_ZERO_DIVISION
            assert me.clock[1].item() == me.clock_val
        else:
            assert res is not None and olerp.bits_equal(got, exp) and c.status == 0


OPEN = {
    "3-outside-peer": [(0, 3), (1, 3), (2, 0)],
    "4-pairs-and-outside": [(0, 1), (1, 0), (2, 4), (3, 4)],
    "5-outside-peers": [(0, 5), (1, 6), (2, 5), (3, 0), (4, 6)],
}


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("name", sorted(OPEN))
def test_open_groups_vs_oracle(dtype, name):
    """Entries whose reads overlap while some peer is outside the dispatch (a learner that did not
    fetch this round) still run as one group: the outside slots are extra sources with no output.
    Each entry is bit-exact with the C oracle, and the outside learners' slots stay untouched."""
    picks = OPEN[name]
    L = 1 + max(max(a, b) for a, b in picks)
    rng = np.random.default_rng(31 + len(name))
    n = 8 * 64 * 4 * 2 + 4097
    ls = [Learner(n, dtype, rng, 1.0 + 0.25 * i, 0.2 + 0.1 * i) for i in range(L)]
    for got, exp, _, me in _run(ls, picks, dtype):
        assert olerp.bits_equal(got, exp)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_more_than_eight_sources_keep_the_xcd_grouped_batch(dtype):
    """Six entries with five distinct outside peers (eleven buffers read, one peer read twice):
    beyond the group kernel's eight sources, so the batch runs the XCD-grouped span order -- each
    entry bit-exact with the C oracle."""
    rng = np.random.default_rng(41)
    n = 8 * 64 * 4 * 2 + 77
    ls = [Learner(n, dtype, rng, 1.0 + 0.25 * i, 0.2 + 0.1 * i) for i in range(11)]
    picks = [(0, 6), (1, 7), (2, 8), (3, 9), (4, 10), (5, 6)]
    for got, exp, _, me in _run(ls, picks, dtype):
        assert olerp.bits_equal(got, exp)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("picks", [[(0, 1), (2, 1)], [(0, 1), (1, 2)], [(1, 0), (0, 1)]],
                         ids=["same-peer", "chain", "mutual-reversed"])
def test_two_entries_sharing_a_read(dtype, picks):
    """Two entries that share a read without being a mutual pair (both pick the same peer; one's
    peer is the other's parameters) run as a group of three sources (k_lerp_group); the mutual
    pair given in the other order takes k_lerp_pair: each bit-exact with the C oracle."""
    rng = np.random.default_rng(17)
    n = 8 * 64 * 4 * 5 + 4097
    ls = [Learner(n, dtype, rng, 1.5 + i, 0.3 + 0.2 * i) for i in range(3)]
    for got, exp, _, me in _run(ls, picks, dtype):
        assert olerp.bits_equal(got, exp)


def test_pair_with_a_zero_division_entry():
    """Loss interpolation with loss + peer loss == 0 for one side of a pair (the reference's
    ZeroDivisionError, interpolation.py:31-33): that entry copies its parameters into its next
    slot unchanged and keeps its clock; its partner averages normally."""
    rng = np.random.default_rng(9)
    ls = [Learner(70_001, "f32", rng, 2.0, 0.0), Learner(70_001, "f32", rng, 3.0, 0.0)]
    out = _run(ls, [(0, 1), (1, 0)], "f32", method="loss", losses=[0.0, 0.4])
    (got0, exp0, res0, me0), (got1, exp1, res1, _) = out
    assert res0 is None and olerp.bits_equal(got0, me0.host)
    c0 = _lib.Coef.from_buffer_copy(me0.coef.cpu().numpy().tobytes())
    assert c0.status == _lib.STATUS_ZERO_DIVISION and me0.clock[1].item() == 2.0     # the clock unchanged
    assert res1 is not None and olerp.bits_equal(got1, exp1)


def test_resident_gossip_of_two_learners_matches_oracle(tmp_path):
    """The N=1 bench's round: two resident learners, each the other's only peer, batched -- every
    round a mutual pair -- 20 rounds with a step after each update_wait, against
    oracle/gossip.py (train_after_wait) bit for bit."""
    names = ["p0", "p1"]
    cfg = tmp_path / "pair.yaml"
    lines = ["- nodes:"] + ["  - {name: %s, host: localhost, port: %d}" % (nm, 47100 + i) for i, nm in enumerate(names)]
    lines += ["- fetch_probability: 1", "- timeout_ms: 2500", "- interpolation: clock", "- divergence_threshold: 0",
              "- constant: { value: 0.5 }", "- clock: 0", "- loss: 0"]
    cfg.write_text("\n".join(lines) + "\n")
    rng = np.random.default_rng(21)
    n, T = 3 * 8 * 64 * 4 + 77, 20
    init = rng.standard_normal((2, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, 2, n))).astype(np.float32)
    send = [[1.0 + g + r for g in range(2)] for r in range(T)]
    wait = [[0.5 + g + r for g in range(2)] for r in range(T)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, 1.0, [5, 6], train_after_wait=True)
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=5 + g, group=group) for g in range(2)]
    for g in range(2):
        conns[g].make_resident(torch.from_numpy(init[g]).to(DEV))
    for r in range(T):
        for g in range(2):
            conns[g].update_send(conns[g].parameters, send[r][g])
        res = DpwaConnection.update_wait_average_many(conns, [c.parameters for c in conns], wait[r])
        for g in range(2):
            assert res[g][0] is not None and res[g][0].peer == names[1 - g]
            assert olerp.bits_equal(conns[g].parameters.cpu().numpy(), exp["params"][r, g]), (r, g)
            assert conns[g].clock == exp["clocks"][r, g]
        for g in range(2):
            conns[g].parameters.add_(torch.from_numpy(deltas[r, g]).to(DEV))
    for c in conns:
        c.close()
