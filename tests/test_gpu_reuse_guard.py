"""The adapter's reuse guard: with write-through snapshots, an update_send whose parameters'
version counters did not move publishes the snapshot the last average wrote -- unless the
device check of sampled words finds the parameters changed (a write through ``param.data``,
which no version counter sees).  The reference always publishes the parameters as they are at
update_send (pytorch.py:49-53), so the learners' trajectories must equal the oracle's, which
folds every write into the parameters before the next publish."""
import numpy as np
import pytest
import torch

from dpwa_amd import DpwaPyTorchAdapter
from dpwa_amd.group import LocalGroup
from oracle import lerp as olerp
from tests.helpers import guard_period, guard_words
from tests.test_gpu_gossip import DEV, Net, load_flat, write_cfg

pytestmark = pytest.mark.gpu


def _run(tmp_path, mode, n=100_032, T=5):
    """Two learners averaging with constant 0.5 every round; after each update_wait, `mode`
    writes through param.data: 'dense' (every element), 'first' / 'last' (one element: the
    payload's first / last 16-B word, both always sampled; n is a multiple of the flat
    buffer's 64-element alignment, so the parameter ends where the payload does), 'none'.
    reuse_guard is off for 'unguarded' (dense)."""
    rng = np.random.default_rng(21)
    G = 2
    names = ["a", "b"]
    init = rng.standard_normal((G, n)).astype(np.float32)
    cfg = tmp_path / ("guard_%s.yaml" % mode)
    write_cfg(cfg, names, 1.0, "constant", 0.0, 0.5)
    group = LocalGroup()
    nets, adapters = [], []
    for g in range(G):
        net = Net([(n,)]).to(DEV)
        load_flat(net, init[g])
        nets.append(net)
        adapters.append(DpwaPyTorchAdapter(net, names[g], str(cfg), seed=5 + g, group=group, write_through=True,
                                           reuse_guard=mode != "unguarded"))
    params = init.copy()
    for r in range(T):
        for g in range(G):
            adapters[g].update_send(1.0)
        snaps = [params[g].copy() for g in range(G)]
        for g in range(G):
            adapters[g].update_wait(1.0)
            params[g] = olerp.lerp_f32(params[g], snaps[1 - g], 0.5)
        for g in range(G):
            bump = np.zeros(n, np.float32)
            if mode in ("dense", "unguarded"):
                bump[:] = (0.25 * rng.standard_normal(n)).astype(np.float32)
            elif mode == "first":
                bump[0] = 1.5
            elif mode == "last":
                bump[-1] = -2.5
            if mode != "none":
                with torch.no_grad():
                    nets[g].p0.data.add_(torch.from_numpy(bump).to(DEV))    # no version counter moves
                params[g] = np.add(params[g], bump, dtype=np.float32)
    torch.cuda.synchronize()
    same = [olerp.bits_equal(nets[g].p0.detach().cpu().numpy(), params[g]) for g in range(G)]
    hits = [a.reuse_guard_hits for a in adapters]
    for a in adapters:
        a.connection.close()
    return same, hits, T


@pytest.mark.parametrize("mode", ["dense", "first", "last"])
def test_reuse_guard_catches_writes_through_param_data(tmp_path, mode):
    same, hits, T = _run(tmp_path, mode)
    assert all(same), same
    assert hits == [T - 1, T - 1], hits       # every publish after the first reused, and was caught


def test_reuse_guard_stays_quiet_without_writes(tmp_path):
    same, hits, _ = _run(tmp_path, "none")
    assert all(same), same
    assert hits == [0, 0], hits


def test_without_the_guard_peers_get_the_stale_snapshot(tmp_path):
    """The hazard the guard closes: the same loop with the guard off diverges from the oracle."""
    same, hits, _ = _run(tmp_path, "unguarded")
    assert not any(same), same
    assert hits == [0, 0], hits


def test_reuse_guard_compares_the_tail_bytes(tmp_path):
    """Connection level, an odd element count (payload not a multiple of 16 bytes): a write to
    the last element, which lies in the tail bytes, makes the reusing publish a full one."""
    import ctypes

    from dpwa_amd import DpwaConnection, _lib
    n, T = 100_003, 4
    names = ["a", "b"]
    cfg = tmp_path / "tail.yaml"
    write_cfg(cfg, names, 1.0, "constant", 0.0, 0.5)
    rng = np.random.default_rng(4)
    init = rng.standard_normal((2, n)).astype(np.float32)
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=5 + g, group=group) for g in range(2)]
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(2)]
    params = init.copy()
    for r in range(T):
        for g in range(2):
            conns[g].update_send(flats[g], 1.0, reuse_snapshot=r > 0)
            if r == 0:
                _lib.call("dpwa_learner_set_reuse_guard", conns[g]._learner.handle, 1)
        snaps = [params[g].copy() for g in range(2)]
        for g in range(2):
            conns[g].update_wait_average(flats[g], 1.0, write_through=True)
            params[g] = olerp.lerp_f32(params[g], snaps[1 - g], 0.5)
        flats[0][-1] += 3.0                     # learner a only, behind the caller's assertion
        params[0][-1] = np.float32(params[0][-1] + np.float32(3.0))
    torch.cuda.synchronize()
    for g in range(2):
        assert olerp.bits_equal(flats[g].cpu().numpy(), params[g]), g
    hits = []
    for c in conns:
        h = ctypes.c_uint32()
        _lib.call("dpwa_learner_reuse_guard_hits", c._learner.handle, ctypes.byref(h))
        hits.append(h.value)
        c.close()
    assert hits == [T - 1, 0], hits


def _sparse_round(tmp_path, write_through):
    """Learner a writes ONE element through param.data between update_wait and update_send, at a
    16-B word the guard does not sample at that publish (n16 = 25,008 words, samples every ~6.1
    words, moved by the generation: the second publish compares words 2, 8, 14, ... -- word 3 is
    not one of them).  Learner b averages with constant 1.0, so after the next round b's
    parameters ARE the snapshot a served.  Returns (b's element, the written value, a's element
    before the write, reuse guard hits of a)."""
    n = 100_032
    assert 3 not in guard_words(n * 4 // 16, 2)
    rng = np.random.default_rng(31)
    init = rng.standard_normal((2, n)).astype(np.float32)
    cfg = tmp_path / ("sparse_%d.yaml" % write_through)
    write_cfg(cfg, ["a", "b"], 1.0, "constant", 0.0, 1.0)
    group = LocalGroup()
    nets, ads = [], []
    for g, nm in enumerate(("a", "b")):
        net = Net([(n,)]).to(DEV)
        load_flat(net, init[g])
        nets.append(net)
        ads.append(DpwaPyTorchAdapter(net, nm, str(cfg), seed=40 + g, group=group, write_through=write_through))
    for ad in ads:
        ad.update_send(1.0)
    for ad in ads:
        ad.update_wait(1.0)
    k = 3 * 4 + 1                          # an fp32 element of 16-B word 3 (not sampled)
    before = float(nets[0].p0.detach()[k].item())
    with torch.no_grad():
        nets[0].p0.data[k] = 123.25        # in place through .data: no version counter moves
    for ad in ads:
        ad.update_send(1.0)
    for ad in ads:
        ad.update_wait(1.0)
    got = float(nets[1].p0.detach()[k].item())
    hits = ads[0].reuse_guard_hits
    for ad in ads:
        ad.connection.close()
    return got, 123.25, before, hits


def test_sparse_data_write_missing_the_samples_is_stale_under_write_through(tmp_path):
    """The documented limit of the write-through default (adapter docstring, README quick-start):
    a sparse write through param.data between update_wait and update_send that changes none of the
    guard's sampled words is NOT in the next snapshot -- the peer averages with the value before
    the write (the reference would have published it, pytorch.py:49-53); with write_through=False
    every publish copies the parameters and the peer gets the written value."""
    got, written, before, hits = _sparse_round(tmp_path, True)
    assert hits == 0 and got == before and got != written
    got, written, before, hits = _sparse_round(tmp_path, False)
    assert got == written


def test_rehomed_parameter_warns_once(tmp_path, caplog):
    """A parameter re-homed through param.data (``p.data = ...``) is folded back into the flat buffer
    and published in full, and the write-through adapter warns once -- while its guard has caught
    nothing -- where such loops can meet stale snapshots (the previous test's case)."""
    import logging
    n = 4096
    cfg = tmp_path / "rehome.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "constant", 0.0, 0.5)
    group = LocalGroup()
    nets, ads = [], []
    for g, nm in enumerate(("a", "b")):
        net = Net([(n,)]).to(DEV)
        nets.append(net)
        ads.append(DpwaPyTorchAdapter(net, nm, str(cfg), seed=60 + g, group=group))
    with caplog.at_level(logging.WARNING, logger="dpwa_amd.adapters.pytorch"):
        for r in range(3):
            nets[0].p0.data = torch.full((n,), float(r), device=DEV)     # re-homed every round
            for ad in ads:
                ad.update_send(1.0)
            for ad in ads:
                ad.update_wait(1.0)
    warned = [rec for rec in caplog.records if "re-homed" in rec.getMessage()]
    assert len(warned) == 1 and "write_through=False" in warned[0].getMessage()
    for ad in ads:
        ad.connection.close()


def test_reuse_guard_rotation_catches_a_fixed_unsampled_word(tmp_path):
    """The guard's samples move with the publish generation (kernels.hip guard_offset), so a loop
    that writes the same word through param.data every round -- a word the first guarded publish
    does not sample -- is caught exactly at the publishes whose samples cover it, the first within
    W = ceil((n16-1)/4095) publishes (7 here).  Round r's publish is generation r+1; each caught
    publish copies the parameters in full, so the next round starts from an equal snapshot."""
    n = 100_032
    n16 = n * 4 // 16
    W = guard_period(n16)
    w = next(x for x in range(1, n16) if x not in guard_words(n16, 2))
    k = w * 4 + 1
    cfg = tmp_path / "rotate.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "constant", 0.0, 0.5)
    group = LocalGroup()
    rng = np.random.default_rng(9)
    nets, ads = [], []
    for g, nm in enumerate(("a", "b")):
        net = Net([(n,)]).to(DEV)
        load_flat(net, rng.standard_normal(n).astype(np.float32))
        nets.append(net)
        ads.append(DpwaPyTorchAdapter(net, nm, str(cfg), seed=80 + g, group=group, write_through=True))
    got, want = [], []
    for r in range(2 * W + 1):
        before = ads[0].reuse_guard_hits
        for ad in ads:
            ad.update_send(1.0)
        got.append(ads[0].reuse_guard_hits - before)
        want.append(int(r >= 1 and w in guard_words(n16, r + 1)))
        for ad in ads:
            ad.update_wait(1.0)
        with torch.no_grad():
            nets[0].p0.data[k] += 1.0          # the same element every round, no version counter moves
    for ad in ads:
        ad.connection.close()
    assert got == want, (got, want)
    first = want.index(1)
    assert 1 <= first <= W, (first, W)
    assert sum(want) >= 2                    # and again one period later


def test_reuse_guard_on_unaligned_parameters(tmp_path):
    """Connection level, parameters that start 4 bytes past a 16-B boundary (a view into a larger
    tensor): the guard takes its bytewise form (k_guard_publish_bytes) -- writes to the first
    element (always compared) and to the last one (the tail bytes) make the reusing publish copy
    what changed, and the trajectories equal the oracle's."""
    import ctypes

    from dpwa_amd import DpwaConnection, _lib
    n, T = 100_003, 4
    names = ["a", "b"]
    cfg = tmp_path / "unaligned.yaml"
    write_cfg(cfg, names, 1.0, "constant", 0.0, 0.5)
    rng = np.random.default_rng(8)
    init = rng.standard_normal((2, n)).astype(np.float32)
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=7 + g, group=group) for g in range(2)]
    bases = [torch.zeros(n + 1, device=DEV) for _ in range(2)]
    flats = [bases[g][1:] for g in range(2)]
    for g in range(2):
        flats[g].copy_(torch.from_numpy(init[g]))
        assert flats[g].data_ptr() % 16 == 4
    params = init.copy()
    for r in range(T):
        for g in range(2):
            conns[g].update_send(flats[g], 1.0, reuse_snapshot=r > 0)
            if r == 0:
                _lib.call("dpwa_learner_set_reuse_guard", conns[g]._learner.handle, 1)
        snaps = [params[g].copy() for g in range(2)]
        for g in range(2):
            conns[g].update_wait_average(flats[g], 1.0, write_through=True)
            params[g] = olerp.lerp_f32(params[g], snaps[1 - g], 0.5)
        flats[0][0] += 1.5                      # the first element: always compared
        params[0][0] = np.float32(params[0][0] + np.float32(1.5))
        flats[1][-1] -= 2.0                     # the last element: the tail bytes
        params[1][-1] = np.float32(params[1][-1] - np.float32(2.0))
    torch.cuda.synchronize()
    for g in range(2):
        assert olerp.bits_equal(flats[g].cpu().numpy(), params[g]), g
    hits = []
    for c in conns:
        h = ctypes.c_uint32()
        _lib.call("dpwa_learner_reuse_guard_hits", c._learner.handle, ctypes.byref(h))
        hits.append(h.value)
        c.close()
    assert hits == [T - 1, T - 1], hits


def test_reuse_guard_copies_the_chunks_whose_sample_differs(tmp_path):
    """The one-launch guard copies per chunk (kernels.hip k_guard_publish): learner a writes two
    elements through param.data -- one in a word its next publish samples, one in another chunk's
    unsampled word.  Learner b averages with constant 1.0, so its parameters become the snapshot a
    served: the sampled write reaches b, the unsampled one is not in that snapshot (it would be
    once its chunk's rotating sample reaches it, tests above)."""
    from tests.helpers import guard_chunk
    n = 100_032
    n16 = n * 4 // 16
    gen = 2                                          # a's second publish is the guarded one
    words = sorted(guard_words(n16, gen))
    x = words[len(words) // 2]                       # sampled at gen 2
    cx = guard_chunk(n16, x)[0]
    y = next(w for w in range(n16 // 4, n16) if w not in guard_words(n16, gen) and guard_chunk(n16, w)[0] != cx)
    kx, ky = x * 4 + 2, y * 4 + 1
    rng = np.random.default_rng(41)
    init = rng.standard_normal((2, n)).astype(np.float32)
    cfg = tmp_path / "chunks.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "constant", 0.0, 1.0)
    group = LocalGroup()
    nets, ads = [], []
    for g, nm in enumerate(("a", "b")):
        net = Net([(n,)]).to(DEV)
        load_flat(net, init[g])
        nets.append(net)
        ads.append(DpwaPyTorchAdapter(net, nm, str(cfg), seed=50 + g, group=group, write_through=True))
    for ad in ads:
        ad.update_send(1.0)
    for ad in ads:
        ad.update_wait(1.0)
    before_y = float(nets[0].p0.detach()[ky].item())
    with torch.no_grad():
        nets[0].p0.data[kx] = 77.5
        nets[0].p0.data[ky] = -33.25
    for ad in ads:
        ad.update_send(1.0)
    for ad in ads:
        ad.update_wait(1.0)
    got_x = float(nets[1].p0.detach()[kx].item())
    got_y = float(nets[1].p0.detach()[ky].item())
    hits = ads[0].reuse_guard_hits
    for ad in ads:
        ad.connection.close()
    assert hits == 1
    assert got_x == 77.5
    assert got_y == before_y and got_y != -33.25


@pytest.mark.parametrize("n", [3, 5, 64, 1000])
def test_reuse_guard_on_tiny_models(tmp_path, n):
    """Models below one 16-B word, at a few words and below 4,096 words (every word its own
    chunk): dense writes through param.data are caught at every reusing publish and the
    trajectories equal the oracle's."""
    same, hits, T = _run(tmp_path, "dense", n=n, T=4)
    assert all(same), same
    assert hits == [T - 1, T - 1], hits


@pytest.mark.parametrize("mode", ["dense", "sampled", "unsampled"])
def test_reuse_guard_bf16(tmp_path, mode):
    """bf16 parameters (100,003 elements, padded by the flat buffer to 256 B) through the
    write-through adapter with the guard on, two learners at constant 0.5: dense writes through
    param.data every round give the torch-eager bf16 oracle's trajectories; a write to a word the
    next publish samples reaches the peer at once (its chunk is copied); a write to a word it
    does not sample is not in that publish's snapshot (its chunk's sampled word is elsewhere), and
    the peer averages the old value -- bit for bit as the oracle given that snapshot."""
    from tests.test_gpu_kernels import from_u16, to_u16
    n = 100_003
    rng = np.random.default_rng(17)
    init = olerp.f32_to_bf16(rng.standard_normal((2, n)).astype(np.float32))
    cfg = tmp_path / ("bf16_%s.yaml" % mode)
    write_cfg(cfg, ["a", "b"], 1.0, "constant", 0.0, 0.5)
    group = LocalGroup()
    nets, ads = [], []
    for g, nm in enumerate(("a", "b")):
        net = Net([(n,)], dtype=torch.bfloat16).to(DEV)
        with torch.no_grad():
            net.p0.copy_(from_u16(init[g]))
        nets.append(net)
        ads.append(DpwaPyTorchAdapter(net, nm, str(cfg), seed=60 + g, group=group, write_through=True))
    n16 = ads[0].flat.numel * 2 // 16          # the flat buffer pads the parameter to 256 B
    params = [init[0].copy(), init[1].copy()]
    T = 4
    for r in range(T):
        for ad in ads:
            ad.update_send(1.0)
        snaps = [params[0].copy(), params[1].copy()]
        for g, ad in enumerate(ads):
            ad.update_wait(1.0)
            params[g] = olerp.lerp_bf16(params[g], snaps[1 - g], 0.5)
        torch.cuda.synchronize()
        for g in range(2):
            assert olerp.bits_equal(to_u16(nets[g].p0.detach()), params[g]), (mode, r, g)
        if mode == "dense":
            bump = olerp.f32_to_bf16((0.25 * rng.standard_normal((2, n))).astype(np.float32))
            for g in range(2):
                new = olerp.f32_to_bf16(olerp.bf16_to_f32(params[g]) + olerp.bf16_to_f32(bump[g]))
                with torch.no_grad():
                    nets[g].p0.data.copy_(from_u16(new))        # through .data: no version counter moves
                params[g] = new
        elif r == 0:
            gen = 2                                              # a's next (guarded) publish
            words = guard_words(n16, gen)
            w = (sorted(words)[len(words) // 2] if mode == "sampled"
                 else next(x for x in range(n16 // 2, n // 8) if x not in words))
            k = w * 8 + 3
            old = float(nets[0].p0.detach()[k].item())
            with torch.no_grad():
                nets[0].p0.data[k] = 64.0
            new = params[0].copy()
            new[k] = olerp.f32_to_bf16(np.array([64.0], np.float32))[0]
            if mode == "sampled":
                params[0] = new                                  # the publish takes it: b sees it
            else:
                # a's own parameters hold the write; its snapshot does not (b averages the old value)
                ads_snapshot_old = params[0].copy()
                params[0] = new
                for ad in ads:
                    ad.update_send(1.0)
                snaps = [ads_snapshot_old, params[1].copy()]
                for g, ad in enumerate(ads):
                    ad.update_wait(1.0)
                    params[g] = olerp.lerp_bf16(params[g], snaps[1 - g], 0.5)
                torch.cuda.synchronize()
                for g in range(2):
                    assert olerp.bits_equal(to_u16(nets[g].p0.detach()), params[g]), (mode, "after", g)
                assert old != 64.0
                break
    hits = ads[0].reuse_guard_hits
    for ad in ads:
        ad.connection.close()
    if mode == "dense":
        assert hits == T - 1
    elif mode == "sampled":
        assert hits == 1
    else:
        assert hits == 0
