"""Resident parameters (dpwa_learner_set_resident, include/dpwa_hip.h): a learner's parameters
live in its own two snapshot slots, publishes move no bytes and every average reads the
published slot and writes the other one.  That needs the loop order update_send, update_wait,
training step -- NOT the reference's README order (README.md:18-29, main.py:130-145: update_send,
step, update_wait), which trains while peers read the snapshot and keeps the write-through form.
In the resident order the rounds must match the reference driven that way
(tests/golden/gossip_step_after_wait.*, via oracle/gossip.py train_after_wait) -- parameters,
clocks and peers bit-exact, snapshots served as they were at update_send -- whether the averages
run one by one or batched, with rounds that have no fetch (fetch_probability < 1), and through
the adapter; a write in the send -> wait window is refused."""
import ctypes

import numpy as np
import pytest
import torch

from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter, _lib
from dpwa_amd.group import LocalGroup
from oracle import gossip as ogossip
from oracle import lerp as olerp
from tests.helpers import guard_period, guard_words
from tests.test_gpu_kernels import from_u16, to_u16

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _write_cfg(path, names, fp, interp, threshold=0):
    lines = ["- nodes:"] + ["  - {name: %s, host: localhost, port: %d}" % (n, 47000 + i) for i, n in enumerate(names)]
    lines += ["- fetch_probability: %r" % fp, "- timeout_ms: 2500", "- interpolation: %s" % interp,
              "- divergence_threshold: %r" % threshold, "- constant: { value: 0.5 }", "- clock: 0", "- loss: 0"]
    path.write_text("\n".join(lines) + "\n")


def _case(G, n, T, dtype, seed):
    rng = np.random.default_rng(seed)
    init32 = rng.standard_normal((G, n)).astype(np.float32)
    d32 = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    if dtype == torch.float32:
        return init32, d32, (lambda a: torch.from_numpy(a).to(DEV)), (lambda t: t.cpu().numpy()), {}
    return (olerp.f32_to_bf16(init32), olerp.f32_to_bf16(d32), from_u16, to_u16,
            dict(lerp=olerp.lerp_bf16, add=ogossip.add_bf16))


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_resident_rounds_match_oracle(tmp_path, dtype, batched):
    """Four co-resident resident learners, clock interpolation, fetch_probability 0.7 (rounds
    without a fetch relocate the parameters), 14 rounds, ragged size: after every update_wait
    the resident tensor holds oracle/gossip.py's parameters bit for bit, the clocks and peers
    match, and the tensor alternates between the learner's two slots."""
    G, n, T, fp = 4, 40_009, 14, 0.7
    names = ["r%d" % g for g in range(G)]
    cfg = tmp_path / "res.yaml"
    _write_cfg(cfg, names, fp, "clock")
    init, deltas, to_dev, to_np, kw = _case(G, n, T, dtype, 13)
    send = [[1.0 + 0.1 * g + r for g in range(G)] for r in range(T)]
    wait = [[0.9 + 0.1 * g + r for g in range(G)] for r in range(T)]
    seeds = [310 + g for g in range(G)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, fp, seeds, train_after_wait=True,
                           **kw)
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
    params = [conns[g].make_resident(to_dev(init[g])) for g in range(G)]
    homes = [set() for _ in range(G)]
    no_fetch = 0
    for r in range(T):
        for g in range(G):
            conns[g].update_send(conns[g].parameters, send[r][g])
        if batched:
            res = DpwaConnection.update_wait_average_many(conns, [c.parameters for c in conns], wait[r])
        else:
            res = [conns[g].update_wait_average(conns[g].parameters, wait[r][g]) for g in range(G)]
        for g in range(G):
            params[g] = conns[g].parameters
            homes[g].add(params[g].data_ptr())
            no_fetch += res[g][0] is None
            assert olerp.bits_equal(to_np(params[g]), exp["params"][r, g]), (r, g)
            assert conns[g].clock == exp["clocks"][r, g], (r, g)
            want = exp["picks"][r][g][-1] if exp["picks"][r][g] else None
            assert (res[g][0].peer if res[g][0] is not None else None) == want, (r, g)
        for g in range(G):      # the training step, after update_wait
            params[g].add_(to_dev(deltas[r, g]))
    assert no_fetch > 0                                   # the relocation path ran
    assert all(len(h) == 2 for h in homes)
    for c in conns:
        c.close()


def _served(conn):
    """The latest published snapshot, read from the host (what RxThread would send)."""
    n = conn._learner.numel
    out = np.empty(n, np.float32)
    hdr = ctypes.create_string_buffer(256)
    v = ctypes.c_uint64()
    _lib.call("dpwa_learner_read_snapshot", conn._learner.handle, hdr, ctypes.c_void_p(out.ctypes.data), n * 4,
              ctypes.byref(v))
    return torch.from_numpy(out).to(DEV), v.value


def test_resident_snapshot_is_the_update_send_state(tmp_path):
    """What a peer reads is the parameters as they were at update_send, although the publisher
    averages right after: the served snapshot equals the parameters at update_send before and
    after the round's averages, and each average is pytorch.py:68 over the two sent states."""
    G, n, T = 2, 70_001, 6
    names = ["s0", "s1"]
    cfg = tmp_path / "snap.yaml"
    _write_cfg(cfg, names, 1.0, "constant")
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=20 + g, group=group) for g in range(G)]
    for g in range(G):
        conns[g].make_resident(torch.randn(n, device=DEV, generator=torch.Generator(device=DEV).manual_seed(g)))
    for r in range(T):
        sent = []
        for g in range(G):
            sent.append(conns[g].parameters.clone())
            conns[g].update_send(conns[g].parameters, 1.0)
        for g in range(G):
            snap, v = _served(conns[g])
            assert v == r + 1 and torch.equal(snap, sent[g]), (r, g)
        res = DpwaConnection.update_wait_average_many(conns, [c.parameters for c in conns], [1.0, 1.0])
        for g in range(G):
            payload, _ = res[g]
            assert payload is not None
            snap, v = _served(conns[g])                           # the average left it alone
            assert v == r + 1 and torch.equal(snap, sent[g]), (r, g)
            expect = (0.5 * sent[1 - g]) + (0.5 * sent[g])        # pytorch.py:68 in torch, fp32
            assert torch.equal(conns[g].parameters, expect), (r, g)
        for g in range(G):
            conns[g].parameters.mul_(0.999)
    for c in conns:
        c.close()


def test_resident_zero_division_round_keeps_parameters(tmp_path):
    """Loss interpolation with loss + peer loss == 0 (the reference's ZeroDivisionError,
    interpolation.py:31-33): the no-op average still moves the parameters into the next slot
    unchanged, and the error is raised at the next call as in the other forms."""
    names = ["z0", "z1"]
    cfg = tmp_path / "zd.yaml"
    _write_cfg(cfg, names, 1.0, "loss")
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=60 + g, group=group) for g in range(2)]
    for g in range(2):
        conns[g].make_resident(torch.full((4099,), float(g + 1), device=DEV))
    for g in range(2):
        conns[g].update_send(conns[g].parameters, 0.0)
    before = [c.parameters.clone() for c in conns]
    ptrs = [c.parameters.data_ptr() for c in conns]
    for g in range(2):
        conns[g].update_wait_average(conns[g].parameters, 0.0)
    for g in range(2):
        assert conns[g].parameters.data_ptr() != ptrs[g]
        assert torch.equal(conns[g].parameters, before[g])
    torch.cuda.synchronize()
    with pytest.raises(ZeroDivisionError):
        conns[0].update_send(conns[0].parameters, 1.0)
    for c in conns:
        c.close()


def test_resident_misuse_is_refused(tmp_path):
    """A resident node publishes and averages only the resident tensor; set_resident only before
    the first publish; the split update_wait (factor then lerp) is refused."""
    names = ["m0", "m1"]
    cfg = tmp_path / "mis.yaml"
    _write_cfg(cfg, names, 1.0, "constant")
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=70 + g, group=group) for g in range(2)]
    other = torch.zeros(1000, device=DEV)
    conns[0].make_resident(torch.ones(1000, device=DEV))
    conns[1].update_send(torch.ones(1000, device=DEV), 1.0)
    with pytest.raises(_lib.DpwaError):
        conns[1].make_resident(torch.ones(1000, device=DEV))          # after its first publish
    with pytest.raises(_lib.DpwaError):
        conns[0].update_send(other, 1.0)                               # not the resident tensor
    conns[0].update_send(conns[0].parameters, 1.0)
    with pytest.raises(_lib.DpwaError):
        conns[0].update_wait(1.0)                                      # split form
    for c in conns:
        c.close()


@pytest.mark.parametrize("many", [False, True])
def test_resident_adapter_matches_write_through(tmp_path, many):
    """DpwaPyTorchAdapter(resident=True) over three small models on one GPU, with an optimizer
    step (SGD with momentum) after every update_wait, gives bit for bit the parameters and clocks
    of the write-through adapter; the parameters are re-pointed into the slots every round and
    the optimizer keeps working on them."""
    names = ["a0", "a1", "a2"]
    cfg = tmp_path / "ad.yaml"
    _write_cfg(cfg, names, 0.8, "clock")
    results = {}
    for mode in ("resident", "write_through"):
        torch.manual_seed(5)
        nets = [torch.nn.Sequential(torch.nn.Linear(7, 33), torch.nn.Tanh(), torch.nn.Linear(33, 5)).to(DEV)
                for _ in names]
        grp = LocalGroup()
        ads = [DpwaPyTorchAdapter(nets[g], names[g], str(cfg), seed=40 + g, group=grp,
                                  resident=mode == "resident") for g in range(3)]
        opts = [torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9) for net in nets]
        gen = torch.Generator(device=DEV).manual_seed(9)
        for r in range(8):
            for g, ad in enumerate(ads):
                ad.update_send(1.0 + g + r)
            if many:
                DpwaPyTorchAdapter.update_wait_many(ads, [0.5 + g + r for g in range(3)])
            else:
                for g, ad in enumerate(ads):
                    ad.update_wait(0.5 + g + r)
            for net, opt in zip(nets, opts):
                opt.zero_grad()
                x = torch.randn(4, 7, device=DEV, generator=gen)
                net(x).square().sum().backward()
                opt.step()
        if mode == "resident":
            home = ads[0].connection.parameters
            p0 = next(nets[0].parameters())
            assert home.data_ptr() <= p0.data_ptr() < home.data_ptr() + home.numel() * 4
        results[mode] = ([torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu() for net in nets],
                         [ad.connection.clock for ad in ads])
        for ad in ads:
            ad.connection.close()
    for a, b in zip(results["resident"][0], results["write_through"][0]):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    assert results["resident"][1] == results["write_through"][1]


def test_resident_pointer_api():
    """dpwa_learner_resident_params: NULL / -1 before set_resident, then slot 0, then the other
    slot after an average; relocate is a no-op when the parameters are in the next slot."""
    cfg = _lib.Interp(_lib.INTERP_CONSTANT, 0, 0.5, 0.0)
    n = 5000
    ls = []
    for _ in range(2):
        h = ctypes.c_void_p()
        _lib.call("dpwa_learner_create", ctypes.byref(h), 0, n, _lib.F32, ctypes.byref(cfg))
        ls.append(h)
    p, k = ctypes.c_void_p(), ctypes.c_int()
    _lib.call("dpwa_learner_resident_params", ls[0], ctypes.byref(p), ctypes.byref(k))
    assert p.value is None and k.value == -1
    init = [torch.full((n,), 1.0 + i, device=DEV) for i in range(2)]
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for i in range(2):
        _lib.call("dpwa_learner_set_resident", ls[i], ctypes.c_void_p(init[i].data_ptr()), s)
    _lib.call("dpwa_learner_resident_params", ls[0], ctypes.byref(p), ctypes.byref(k))
    assert k.value == 0 and p.value
    slot0 = p.value
    _lib.call("dpwa_learner_relocate", ls[0], s)                  # already in the next slot
    _lib.call("dpwa_learner_resident_params", ls[0], ctypes.byref(p), ctypes.byref(k))
    assert k.value == 0 and p.value == slot0
    for i in range(2):
        rp = ctypes.c_void_p()
        _lib.call("dpwa_learner_resident_params", ls[i], ctypes.byref(rp), None)
        _lib.call("dpwa_learner_publish", ls[i], rp, 1.0, None, s)
    _lib.call("dpwa_learner_attach_local", ls[0], 1, ls[1])
    _lib.call("dpwa_learner_fetch", ls[0], 1, 1, _lib.FETCH_ZERO_COPY, s)
    _lib.call("dpwa_learner_average", ls[0], ctypes.c_void_p(slot0), 1.0, None, s)
    _lib.call("dpwa_learner_resident_params", ls[0], ctypes.byref(p), ctypes.byref(k))
    assert k.value == 1 and p.value != slot0
    from dpwa_amd.devview import device_tensor
    got = device_tensor(p.value, n, torch.float32, DEV)
    assert torch.equal(got, torch.full((n,), 1.5, device=DEV))     # 0.5*2 + 0.5*1
    assert torch.equal(device_tensor(slot0, n, torch.float32, DEV), init[0])   # the snapshot, untouched
    torch.cuda.synchronize()
    del got
    for h in ls:
        _lib.call("dpwa_learner_destroy", h)


def test_resident_refuses_a_write_between_send_and_wait(tmp_path):
    """The reference's own order (update_send, optimizer step, update_wait; main.py:130-145) under
    resident=True would serve peers a snapshot being trained: update_wait raises DpwaError naming
    the order instead -- through the adapter (SGD step), the batched adapter call, and the
    connection (an in-place op on conn.parameters) -- and nothing was averaged.  The resident
    order (step after update_wait) keeps working, and so does the write-through adapter in the
    reference order."""
    names = ["v0", "v1"]
    cfg = tmp_path / "win.yaml"
    _write_cfg(cfg, names, 1.0, "constant")
    torch.manual_seed(3)
    for many in (False, True):
        nets = [torch.nn.Sequential(torch.nn.Linear(6, 9), torch.nn.Linear(9, 2)).to(DEV) for _ in names]
        grp = LocalGroup()
        ads = [DpwaPyTorchAdapter(nets[g], names[g], str(cfg), seed=80 + g, group=grp, resident=True)
               for g in range(2)]
        opts = [torch.optim.SGD(n.parameters(), lr=0.1) for n in nets]

        def sgd_step(g):
            opts[g].zero_grad()
            nets[g](torch.randn(3, 6, device=DEV)).sum().backward()
            opts[g].step()

        for r in range(2):      # the resident order works
            for ad in ads:
                ad.update_send(1.0)
            if many:
                DpwaPyTorchAdapter.update_wait_many(ads, [1.0, 1.0])
            else:
                for ad in ads:
                    ad.update_wait(1.0)
            for g in range(2):
                sgd_step(g)
        for ad in ads:
            ad.update_send(1.0)
        before = ads[1].connection.parameters.clone()
        sgd_step(1)                                             # the reference's step position
        with pytest.raises(_lib.DpwaError, match="update_send -> update_wait -> step"):
            if many:
                DpwaPyTorchAdapter.update_wait_many(ads, [1.0, 1.0])
            else:
                ads[0].update_wait(1.0)                          # untouched: averages
                ads[1].update_wait(1.0)
        assert not torch.equal(ads[1].connection.parameters, before)  # the step's write, not an average
        torch.cuda.synchronize()
        for ad in ads:
            ad.connection.close()
    # the connection-level form: an in-place write of the resident tensor in the window
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=90 + g, group=group) for g in range(2)]
    for g in range(2):
        conns[g].make_resident(torch.full((5000,), float(g), device=DEV))
    for c in conns:
        c.update_send(c.parameters, 1.0)
    conns[0].parameters[7:9].mul_(2.0)                         # a view shares the version counter
    with pytest.raises(_lib.DpwaError, match="modified between update_send and update_wait"):
        DpwaConnection.update_wait_average_many(conns, [c.parameters for c in conns], [1.0, 1.0])
    with pytest.raises(_lib.DpwaError):
        conns[0].update_wait_average(conns[0].parameters, 1.0)
    conns[1].update_wait_average(conns[1].parameters, 1.0)     # its own window is clean
    torch.cuda.synchronize()
    for c in conns:
        c.close()


def test_resident_adapter_second_publish_without_wait_follows_the_parameters(tmp_path):
    """Two update_sends with no update_wait between them: the second publish relocates the
    parameters into the slot it publishes (dpwa_learner_relocate), and the adapter re-points
    every parameter there, so the next update_wait averages them where they are and the
    optimizer keeps training the live tensor."""
    names = ["q0", "q1"]
    cfg = tmp_path / "twice.yaml"
    _write_cfg(cfg, names, 1.0, "constant")
    torch.manual_seed(4)
    nets = [torch.nn.Linear(5, 3).to(DEV) for _ in names]
    grp = LocalGroup()
    ads = [DpwaPyTorchAdapter(nets[g], names[g], str(cfg), seed=95 + g, group=grp, resident=True) for g in range(2)]
    for ad in ads:
        ad.update_send(1.0)
    for ad in ads:
        ad.update_wait(1.0)
    ads[0].update_send(1.0)
    home = ads[0].connection.parameters.data_ptr()
    ads[0].update_send(1.0)                                     # again, no average in between
    moved = ads[0].connection.parameters
    assert moved.data_ptr() != home
    for p in nets[0].parameters():
        assert moved.data_ptr() <= p.data_ptr() < moved.data_ptr() + moved.numel() * 4
    ads[1].update_send(1.0)
    peer = ads[1].connection.parameters.clone()
    mine = moved.clone()
    for ad in ads:
        ad.update_wait(1.0)
    want = (0.5 * peer) + (0.5 * mine)                          # pytorch.py:68, fp32
    assert torch.equal(ads[0].connection.parameters, want)
    w = next(nets[0].parameters())
    lo = ads[0].connection.parameters.data_ptr()
    assert lo <= w.data_ptr() < lo + want.numel() * 4
    torch.cuda.synchronize()
    for ad in ads:
        ad.connection.close()


@pytest.mark.parametrize("many", [False, True])
def test_resident_window_guard_catches_data_writes(tmp_path, many):
    """Writes through ``param.data`` in the send -> wait window move no version counter, so
    _check_window cannot see them; the window guard (reuse_guard, on by default) compares the
    published payload's sampled words at update_wait on the device.  These models are smaller than
    4096 16-B words, so every word is sampled and a one-element write is caught: the learner that
    wrote counts the window (window_guard_hits) and its next update_send raises DpwaError without
    publishing; the one after proceeds, and the other learner is untouched.  With
    reuse_guard=False nothing is checked."""
    names = ["w0", "w1"]
    cfg = tmp_path / "wg.yaml"
    _write_cfg(cfg, names, 1.0, "constant")
    torch.manual_seed(6)
    for guard in (True, False):
        nets = [torch.nn.Sequential(torch.nn.Linear(6, 9), torch.nn.Linear(9, 2)).to(DEV) for _ in names]
        grp = LocalGroup()
        ads = [DpwaPyTorchAdapter(nets[g], names[g], str(cfg), seed=70 + g, group=grp, resident=True,
                                  reuse_guard=guard) for g in range(2)]
        opts = [torch.optim.SGD(n.parameters(), lr=0.1) for n in nets]

        def wait_all():
            if many:
                DpwaPyTorchAdapter.update_wait_many(ads, [1.0, 1.0])
            else:
                for ad in ads:
                    ad.update_wait(1.0)

        def steps():
            for g in range(2):
                opts[g].zero_grad()
                nets[g](torch.randn(3, 6, device=DEV)).sum().backward()
                opts[g].step()

        for r in range(3):                  # the resident order, no window written
            for ad in ads:
                ad.update_send(1.0)
            wait_all()
            steps()
        assert [ad.window_guard_hits for ad in ads] == [0, 0]
        for ad in ads:
            ad.update_send(1.0)
        w = list(nets[1].parameters())[2]
        w.data[0, 0] += 1.0                 # one element, through .data: no version counter moves
        wait_all()                          # the version check passes; the device check does not
        steps()
        assert [ad.window_guard_hits for ad in ads] == ([0, 1] if guard else [0, 0])
        ads[0].update_send(1.0)
        if guard:
            with pytest.raises(_lib.DpwaError, match="written between update_send and update_wait"):
                ads[1].update_send(1.0)
        ads[1].update_send(1.0)             # reported once: this publish proceeds
        wait_all()
        steps()
        for ad in ads:
            ad.update_send(1.0)
        wait_all()
        assert [ad.window_guard_hits for ad in ads] == ([0, 1] if guard else [0, 0])
        torch.cuda.synchronize()
        for ad in ads:
            ad.connection.close()


def test_resident_window_guard_samples_and_tail_bytes(tmp_path):
    """The window guard's sampling on a model larger than its 4096 words: ragged bf16
    (100003 elements: 12500 16-B words and 6 tail bytes), connection level with the guard set
    through the C ABI.  A write to the tail bytes or to a word sampled at that publish's
    generation is caught (window_hits grows, the next update_send raises), a write to a word that
    generation's samples miss is not -- the samples move on by one word each publish, so a later
    window covers it (next test) -- and rounds with no write stay clean.  Writes go through a
    second view of the resident memory, so no version counter of conn.parameters moves."""
    from dpwa_amd.devview import device_tensor
    names = ["t0", "t1"]
    cfg = tmp_path / "tail.yaml"
    _write_cfg(cfg, names, 1.0, "constant")
    n = 100_003
    n16 = n * 2 // 16
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=60 + g, group=group) for g in range(2)]
    for g in range(2):
        conns[g].make_resident(torch.randn(n, device=DEV).to(torch.bfloat16))
        _lib.call("dpwa_learner_set_reuse_guard", conns[g]._learner.handle, 1)

    def hits(c):
        h = ctypes.c_uint32()
        _lib.call("dpwa_learner_window_hits", c._learner.handle, ctypes.byref(h))
        return h.value

    def gen(c):
        v = ctypes.c_uint64()
        _lib.call("dpwa_learner_version", c._learner.handle, ctypes.byref(v))
        return v.value

    def round_(write=None):
        for c in conns:
            c.update_send(c.parameters, 1.0)
        if write is not None:
            p = conns[1].parameters
            alias = device_tensor(p.data_ptr(), n, torch.bfloat16, DEV)    # its own version counter
            alias[write(gen(conns[1]))] += 1.0
            del alias
        for c in conns:
            c.update_wait_average(c.parameters, 1.0)

    def sampled(g):
        return sorted(guard_words(n16, g))[1] * 8 + 3                      # inside a word sampled at g

    def unsampled(g):
        return next(w for w in range(1, n16) if w not in guard_words(n16, g)) * 8 + 5

    round_()
    round_()
    assert [hits(c) for c in conns] == [0, 0]
    expect = 0
    for elem, caught in ((lambda g: n - 1, True),                        # a tail byte
                         (sampled, True),
                         (unsampled, False)):
        round_(write=elem)
        expect += caught
        assert hits(conns[1]) == expect and hits(conns[0]) == 0, caught
        conns[0].update_send(conns[0].parameters, 1.0)
        if caught:
            with pytest.raises(_lib.DpwaError, match="written between update_send and update_wait"):
                conns[1].update_send(conns[1].parameters, 1.0)
        conns[1].update_send(conns[1].parameters, 1.0)
        for c in conns:
            c.update_wait_average(c.parameters, 1.0)
        round_()
        assert hits(conns[1]) == expect
    torch.cuda.synchronize()
    for c in conns:
        c.close()


def test_resident_window_guard_rotation_catches_a_fixed_word(tmp_path):
    """A loop that writes the same 16-B word in every send -> wait window (a word the first
    window's samples miss): the window guard's samples move on by one word per publish, so the
    window of publish generation g is caught exactly when the word is among generation g's
    samples -- the first within W = ceil((n16-1)/4095) windows (4 here) -- and each caught window
    makes the next update_send raise once."""
    from dpwa_amd.devview import device_tensor
    names = ["t0", "t1"]
    cfg = tmp_path / "rot.yaml"
    _write_cfg(cfg, names, 1.0, "constant")
    n = 100_003
    n16 = n * 2 // 16
    W = guard_period(n16)
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=90 + g, group=group) for g in range(2)]
    for g in range(2):
        conns[g].make_resident(torch.randn(n, device=DEV).to(torch.bfloat16))
        _lib.call("dpwa_learner_set_reuse_guard", conns[g]._learner.handle, 1)
    v = ctypes.c_uint64()
    _lib.call("dpwa_learner_version", conns[1]._learner.handle, ctypes.byref(v))
    w = next(x for x in range(1, n16) if x not in guard_words(n16, v.value + 1))
    got, want = [], []
    h = ctypes.c_uint32()
    for r in range(2 * W + 1):
        for c in conns:
            try:
                c.update_send(c.parameters, 1.0)
            except _lib.DpwaError:            # the last window was caught: reported once
                c.update_send(c.parameters, 1.0)
        _lib.call("dpwa_learner_version", conns[1]._learner.handle, ctypes.byref(v))
        want.append(int(w in guard_words(n16, v.value)))
        p = conns[1].parameters
        alias = device_tensor(p.data_ptr(), n, torch.bfloat16, DEV)
        alias[w * 8 + 2] += 1.0
        del alias
        for c in conns:
            c.update_wait_average(c.parameters, 1.0)
        _lib.call("dpwa_learner_window_hits", conns[1]._learner.handle, ctypes.byref(h))
        got.append(h.value)
    torch.cuda.synchronize()
    for c in conns:
        c.close()
    assert np.diff([0] + got).tolist() == want, (got, want)
    assert want[0] == 0 and 1 <= want.index(1) <= W and sum(want) >= 2
