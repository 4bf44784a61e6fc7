"""End-to-end parity of the drop-in API on one GPU: G learners in one process
(LocalGroup) replay the reference's own lock-step gossip trajectories
(tests/golden/gossip.*, produced by running the reference adapter + connection +
TxThread), bit for bit: parameters, clocks, factors and peer choices."""
import numpy as np
import pytest
import torch

from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter
from dpwa_amd.group import LocalGroup
from oracle import gossip as ogossip
from oracle import lerp as olerp
from tests.helpers import load_json, load_npz

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


class Net(torch.nn.Module):
    def __init__(self, shapes, dtype=torch.float32):
        super().__init__()
        for i, s in enumerate(shapes):
            self.register_parameter("p%d" % i, torch.nn.Parameter(torch.zeros(s, dtype=dtype)))


def write_cfg(path, names, fp, interp, thr, value):
    lines = ["---", "- nodes:"]
    lines += ["  - {name: %s, host: localhost, port: %d}" % (n, 46000 + i) for i, n in enumerate(names)]
    lines += ["- fetch_probability: %r" % fp, "- timeout_ms: 2500", "- interpolation: %s" % interp,
              "- divergence_threshold: %r" % thr, "- constant: { value: %r }" % (value if value is not None else 0.5),
              "- clock: 0", "- loss: 0"]
    path.write_text("\n".join(lines) + "\n")


def load_flat(net, flat):
    off = 0
    with torch.no_grad():
        for _, p in net.named_parameters():
            n = p.numel()
            p.data.copy_(torch.from_numpy(flat[off:off + n]).view(p.shape))
            off += n


def flat_params(net):
    return np.concatenate([p.detach().cpu().numpy().reshape(-1) for _, p in net.named_parameters()])


def run_gossip(case, z, tmp_path, dtype=torch.float32):
    names = case["names"]
    G = case["G"]
    shapes = [tuple(s) for s in load_json("gossip.json")["shapes"]]
    cfg = tmp_path / ("%s.yaml" % case["key"])
    write_cfg(cfg, names, case["fetch_probability"], case["interpolation"], case["divergence_threshold"],
              case["value"])
    init, deltas = z[case["key"] + "_init"], z[case["key"] + "_deltas"]
    group = LocalGroup()
    nets, adapters = [], []
    for g in range(G):
        net = Net(shapes).to(DEV)
        load_flat(net, init[g])
        nets.append(net)
        adapters.append(DpwaPyTorchAdapter(net, names[g], str(cfg), seed=case["seeds"][g], group=group))
    T = deltas.shape[0]
    out = {"params": np.zeros((T, G, init.shape[1]), np.float32), "clocks": np.zeros((T, G)),
           "factors": np.zeros((T, G)), "picks": [[None] * G for _ in range(T)], "fetching": np.zeros((T, G), bool)}
    for r in range(T):
        for g in range(G):
            adapters[g].update_send(case["send_loss"][r][g])
            out["fetching"][r, g] = adapters[g].connection.fetching
        for g in range(G):
            with torch.no_grad():
                off = 0
                for _, p in nets[g].named_parameters():
                    k = p.numel()
                    p.data.add_(torch.from_numpy(deltas[r, g, off:off + k]).to(DEV).view(p.shape))
                    off += k
        for g in range(G):
            c = adapters[g].connection
            adapters[g].update_wait(case["wait_loss"][r][g])
            fetched = c.last_fetch_peer is not None and out["fetching"][r, g]
            out["picks"][r][g] = [c.last_fetch_peer] if fetched else []
            out["factors"][r, g] = float(c._learner.read_coef().factor) if fetched else 0.0
            out["clocks"][r, g] = c.clock
            out["params"][r, g] = flat_params(nets[g])
    for a in adapters:
        a.connection.close()
    return out


def test_gossip_matches_reference_trajectories(tmp_path):
    meta = load_json("gossip.json")
    z = load_npz("gossip.npz")
    for case in meta["cases"]:
        k = case["key"]
        got = run_gossip(case, z, tmp_path)
        assert np.array_equal(got["fetching"], z[k + "_fetching"]), k
        assert got["picks"] == case["picks"], k
        assert np.array_equal(got["factors"], z[k + "_factors"]), k
        assert np.array_equal(got["clocks"], z[k + "_clocks"]), k
        assert olerp.bits_equal(got["params"], z[k + "_params"]), k


@pytest.mark.parametrize("form", ["resident", "resident-many", "write-through"])
def test_step_after_wait_matches_reference_trajectories(tmp_path, form):
    """The reference driven update_send -> update_wait -> step (tests/golden/gossip_step_after_wait.*:
    G = 3 and 4, clock and loss interpolation, fetch_probability 0.7): the resident adapter (one by
    one and batched) and the write-through adapter replay it bit for bit -- parameters after every
    update_wait, clocks, factors, fetch gates and peers."""
    meta = load_json("gossip_step_after_wait.json")
    z = load_npz("gossip_step_after_wait.npz")
    shapes = [tuple(s) for s in meta["shapes"]]
    for case in meta["cases"]:
        k, names, G = case["key"], case["names"], case["G"]
        cfg = tmp_path / ("%s_%s.yaml" % (k, form))
        write_cfg(cfg, names, case["fetch_probability"], case["interpolation"], case["divergence_threshold"],
                  case["value"])
        init, deltas = z[k + "_init"], z[k + "_deltas"]
        group = LocalGroup()
        nets, ads = [], []
        for g in range(G):
            net = Net(shapes).to(DEV)
            load_flat(net, init[g])
            nets.append(net)
            ads.append(DpwaPyTorchAdapter(net, names[g], str(cfg), seed=case["seeds"][g], group=group,
                                          resident=form.startswith("resident")))
        for r in range(deltas.shape[0]):
            fetching = []
            for g in range(G):
                ads[g].update_send(case["send_loss"][r][g])
                fetching.append(ads[g].connection.fetching)
            assert fetching == list(z[k + "_fetching"][r]), (k, r)
            if form == "resident-many":
                DpwaPyTorchAdapter.update_wait_many(ads, case["wait_loss"][r])
            else:
                for g in range(G):
                    ads[g].update_wait(case["wait_loss"][r][g])
            for g in range(G):
                c = ads[g].connection
                fetched = fetching[g] and c.last_fetch_peer is not None
                assert ([c.last_fetch_peer] if fetched else []) == case["picks"][r][g], (k, r, g)
                factor = float(c._learner.read_coef().factor) if fetched else 0.0
                assert factor == z[k + "_factors"][r, g], (k, r, g)
                assert c.clock == z[k + "_clocks"][r, g], (k, r, g)
                assert olerp.bits_equal(flat_params(nets[g]), z[k + "_params"][r, g]), (k, r, g)
            for g in range(G):          # the training step, after update_wait
                with torch.no_grad():
                    off = 0
                    for _, p in nets[g].named_parameters():
                        n = p.numel()
                        p.add_(torch.from_numpy(deltas[r, g, off:off + n]).to(DEV).view(p.shape))
                        off += n
        for a in ads:
            a.connection.close()


def test_gossip_longer_run_matches_oracle(tmp_path):
    """A longer synthetic run (loss interpolation, divergence threshold, p<1) against the
    oracle's lock-step simulation."""
    rng = np.random.default_rng(9)
    G, n, T = 5, 5000, 30
    names = ["n%d" % g for g in range(G)]
    init = rng.standard_normal((G, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    send = [[float(2 * np.exp(-r / 8) + 0.05 * rng.random()) for _ in range(G)] for r in range(T)]
    wait = [[float(2 * np.exp(-(r + .5) / 8) + 0.05 * rng.random()) for _ in range(G)] for r in range(T)]
    seeds = [77 + g for g in range(G)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "loss", None, 0.5, 0.8, seeds)
    cfg = tmp_path / "long.yaml"
    write_cfg(cfg, names, 0.8, "loss", 0.5, None)
    group = LocalGroup()
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
    for r in range(T):
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g])
        for g in range(G):
            flats[g].add_(torch.from_numpy(deltas[r, g]).to(DEV))
        for g in range(G):
            payload, factor = conns[g].update_wait(wait[r][g])
            if payload is not None:
                conns[g].average(flats[g])
        for g in range(G):
            assert olerp.bits_equal(flats[g].cpu().numpy(), exp["params"][r, g]), (r, g)
            assert conns[g].clock == exp["clocks"][r, g]


def test_loss_tensor_on_device_is_used_without_sync(tmp_path):
    cfg = tmp_path / "t.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "loss", 0.0, None)
    g = LocalGroup()
    a = DpwaConnection("a", str(cfg), seed=1, group=g)
    b = DpwaConnection("b", str(cfg), seed=2, group=g)
    fa = torch.ones(1000, device=DEV)
    fb = torch.zeros(1000, device=DEV)
    a.update_send(fa, torch.tensor(1.0, device=DEV))
    b.update_send(fb, torch.tensor(3.0, device=DEV, dtype=torch.float32))
    payload, factor = a.update_wait(torch.tensor(1.0, device=DEV))
    a.average(fa)
    assert float(factor) == 1.0 / (1.0 + 3.0)          # loss/(loss+peer_loss)
    want = torch.full((1000,), np.float32(0.25) * 0.0 + np.float32(0.75) * 1.0, device=DEV)
    assert torch.equal(fa, want)


def test_zero_division_is_raised_at_next_call(tmp_path):
    cfg = tmp_path / "z.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "loss", 0.0, None)
    g = LocalGroup()
    a = DpwaConnection("a", str(cfg), seed=1, group=g)
    b = DpwaConnection("b", str(cfg), seed=2, group=g)
    fa, fb = torch.ones(64, device=DEV), torch.zeros(64, device=DEV)
    a.update_send(fa, 0.0)
    b.update_send(fb, 0.0)
    a.update_wait(0.0)
    a.average(fa)
    with pytest.raises(ZeroDivisionError):
        a.synchronize()
    assert torch.equal(fa, torch.ones(64, device=DEV))     # the round was a no-op
    assert a.clock == 1.0


def test_peer_not_up_and_no_state_follow_reference_flow_control(tmp_path):
    """Peers that are not constructed yet are refused (score -100, no data); constructed but
    unpublished peers give an empty reply (score +10, pick again)."""
    cfg = tmp_path / "f.yaml"
    write_cfg(cfg, ["a", "b", "c"], 1.0, "constant", 0.0, 0.5)
    g = LocalGroup()
    a = DpwaConnection("a", str(cfg), seed=3, group=g)
    fa = torch.ones(256, device=DEV)
    a.update_send(fa, 1.0)
    payload, factor = a.update_wait(1.0)
    assert payload is None and factor == 0
    assert sorted(a.flow_control_scores().values()) == [900, 1000]
    b = DpwaConnection("b", str(cfg), seed=4, group=g)
    c = DpwaConnection("c", str(cfg), seed=5, group=g)
    fb = torch.zeros(256, device=DEV)
    b.update_send(fb, 1.0)          # c never publishes
    for _ in range(5):
        a.update_send(fa, 1.0)
        payload, factor = a.update_wait(1.0)
        assert payload is not None and payload.peer == "b"
        a.average(fa)
    a.inject_fault("b", "slow")
    a.update_send(fa, 1.0)
    c.update_send(torch.zeros(256, device=DEV), 1.0)
    payload, _ = a.update_wait(1.0)
    assert payload is not None and payload.peer == "c"
    assert a.flow_control_scores()["b"] < 1000
    a.inject_fault("b", "dead")
    a.inject_fault("c", "dead")
    a.update_send(fa, 1.0)
    payload, _ = a.update_wait(1.0)
    assert payload is None and set(a.flow_control_scores().values()) == {None}


def test_cross_stream_ordering(tmp_path):
    """Each learner runs on its own stream and each stream is stalled with a spin kernel
    before it publishes / averages, so any missing RAW/WAR dependency on the snapshot
    slots would read stale or half-written data.  Results must still equal the oracle."""
    rng = np.random.default_rng(4)
    G, n, T = 3, 2_000_003, 6
    names = ["s%d" % g for g in range(G)]
    init = rng.standard_normal((G, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    send = [[1.0 + 0.1 * g + r for g in range(G)] for r in range(T)]
    wait = [[1.5 + 0.1 * g + r for g in range(G)] for r in range(T)]
    seeds = [31 + g for g in range(G)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, 1.0, seeds)
    cfg = tmp_path / "streams.yaml"
    write_cfg(cfg, names, 1.0, "clock", 0.0, None)
    group = LocalGroup()
    streams = [torch.cuda.Stream() for _ in range(G)]
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    dts = [[torch.from_numpy(deltas[r, g]).to(DEV) for g in range(G)] for r in range(T)]
    torch.cuda.synchronize()
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
    for r in range(T):
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                torch.cuda._sleep(2_000_000 * (G - g))      # later learners' streams run ahead
                conns[g].update_send(flats[g], send[r][g])
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                flats[g].add_(dts[r][g])
        for g in reversed(range(G)):
            with torch.cuda.stream(streams[g]):
                torch.cuda._sleep(1_000_000 * g)
                payload, _ = conns[g].update_wait_average(flats[g], wait[r][g])
    torch.cuda.synchronize()
    for g in range(G):
        assert olerp.bits_equal(flats[g].cpu().numpy(), exp["params"][-1, g]), g
        assert conns[g].clock == exp["clocks"][-1, g]


def test_update_wait_without_average_then_continue(tmp_path):
    """update_wait() whose snapshot is never averaged must not block later rounds."""
    cfg = tmp_path / "skip.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "constant", 0.0, 0.5)
    g = LocalGroup()
    a = DpwaConnection("a", str(cfg), seed=1, group=g)
    b = DpwaConnection("b", str(cfg), seed=2, group=g)
    fa, fb = torch.ones(1024, device=DEV), torch.zeros(1024, device=DEV)
    for r in range(4):
        a.update_send(fa, 1.0)
        b.update_send(fb, 1.0)
        pa, _ = a.update_wait(1.0)          # never averaged
        pb, f = b.update_wait(1.0)
        b.average(fb)
        assert pa is not None and pb is not None
    torch.cuda.synchronize()
    assert torch.equal(fa, torch.ones(1024, device=DEV))
    assert a.clock == 4.0    # the clock still follows dpwa.py:150 (factor 0.5 between equal clocks)


def test_full_publish_matches_reference_trajectories(tmp_path):
    """The adapter's default is write-through (the trajectory tests above run it); with
    write_through=False every publish copies the full snapshot -- trajectories are the same
    bits."""
    meta = load_json("gossip.json")
    z = load_npz("gossip.npz")
    case = meta["cases"][1]
    k = case["key"]
    import dpwa_amd.adapters.pytorch as ap
    orig = ap.DpwaPyTorchAdapter.__init__

    def init_wt(self, net, name, cfg, **kw):
        orig(self, net, name, cfg, write_through=False, **kw)

    ap.DpwaPyTorchAdapter.__init__ = init_wt
    try:
        got = run_gossip(case, z, tmp_path)
    finally:
        ap.DpwaPyTorchAdapter.__init__ = orig
    assert np.array_equal(got["clocks"], z[k + "_clocks"])
    assert olerp.bits_equal(got["params"], z[k + "_params"])


def test_write_through_detects_inplace_updates(tmp_path):
    """An optimizer-style in-place update between update_wait and update_send bumps the
    parameter version counters and forces a full publish (peers see the updated values)."""
    rng = np.random.default_rng(12)
    G, n, T = 2, 3000, 6
    names = ["a", "b"]
    init = rng.standard_normal((G, n)).astype(np.float32)
    cfg = tmp_path / "wt.yaml"
    write_cfg(cfg, names, 1.0, "constant", 0.0, 0.5)
    group = LocalGroup()
    nets = []
    adapters = []
    for g in range(G):
        net = Net([(n,)]).to(DEV)
        load_flat(net, init[g])
        nets.append(net)
        adapters.append(DpwaPyTorchAdapter(net, names[g], str(cfg), seed=5 + g, group=group, write_through=True))
    # oracle: the same loop with the post-average update folded into the next round's delta
    deltas = np.zeros((T, G, n), np.float32)
    bumps = (0.5 * rng.standard_normal((T, G, n))).astype(np.float32)
    params = init.copy()
    from oracle.policy import OracleLearner
    L = [OracleLearner(names[g], [names[1 - g]], 1.0, "constant", 0.5, 0.0, 5 + g) for g in range(G)]
    for r in range(T):
        for g in range(G):
            adapters[g].update_send(1.0)
        snaps = [params[g].copy() for g in range(G)]
        for g in range(G):
            L[g].update_send(1.0)
        for g in range(G):
            adapters[g].update_wait(1.0)
            st, pl, _ = L[g].fetch(lambda p: "ok", lambda p: ("payload", {"clock": 1, "loss": 1.0}, None))
            params[g] = olerp.lerp_f32(params[g], snaps[1 - g], 0.5)
        for g in range(G):     # the "optimizer step" placed after update_wait
            with torch.no_grad():
                nets[g].p0.add_(torch.from_numpy(bumps[r, g]).to(DEV))
            params[g] = np.add(params[g], bumps[r, g], dtype=np.float32)
    torch.cuda.synchronize()
    for g in range(G):
        assert olerp.bits_equal(nets[g].p0.detach().cpu().numpy(), params[g]), g
    del deltas


def test_connection_write_through_and_reuse(tmp_path):
    rng = np.random.default_rng(3)
    G, n, T = 3, 100_001, 8
    names = ["x%d" % g for g in range(G)]
    init = rng.standard_normal((G, n)).astype(np.float32)
    deltas = np.zeros((T, G, n), np.float32)
    send = [[1.0] * G for _ in range(T)]
    wait = [[1.0] * G for _ in range(T)]
    seeds = [9, 10, 11]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, 1.0, seeds)
    cfg = tmp_path / "wt2.yaml"
    write_cfg(cfg, names, 1.0, "clock", 0.0, None)
    group = LocalGroup()
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
    for r in range(T):
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g], reuse_snapshot=r > 0)
        for g in range(G):
            conns[g].update_wait_average(flats[g], wait[r][g], write_through=True)
    for g in range(G):
        assert olerp.bits_equal(flats[g].cpu().numpy(), exp["params"][-1, g]), g


def test_kernel_dispatch_timing(tmp_path):
    """dpwa_learner_time_averages / arm_timing / read_average_times: only armed launches are
    timed, the durations are positive, and timing does not change the results."""
    import ctypes
    from dpwa_amd import _lib
    cfg = tmp_path / "t.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "constant", 0.0, 0.5)
    group = LocalGroup()
    n = 1 << 20
    flats = [torch.randn(n, device=DEV), torch.randn(n, device=DEV)]
    want = (0.5 * flats[1] + 0.5 * flats[0]).clone()
    conns = [DpwaConnection(nm, str(cfg), seed=i, group=group) for i, nm in enumerate(["a", "b"])]
    for c, f in zip(conns, flats):
        c.update_send(f, 1.0)
    h = conns[0]._learner.handle
    _lib.call("dpwa_learner_time_averages", h, 4)
    _lib.call("dpwa_learner_arm_timing", h)
    for c, f in zip(conns, flats):
        c.update_wait_average(f, 1.0)
    for r in range(3):                     # unarmed rounds are not timed
        for c, f in zip(conns, flats):
            c.update_send(f, 1.0)
        for c, f in zip(conns, flats):
            c.update_wait_average(f, 1.0)
    buf = (ctypes.c_float * 4)()
    cnt = ctypes.c_int()
    _lib.call("dpwa_learner_read_average_times", h, buf, 4, ctypes.byref(cnt))
    assert cnt.value == 1
    assert 0.0 < buf[0] < 10_000.0
    torch.cuda.synchronize()
    assert torch.equal(flats[0], want) and torch.equal(flats[1], want)   # f = 0.5 fixed point
    _lib.call("dpwa_learner_time_averages", h, 0)
    for c in conns:
        c.close()


@pytest.mark.parametrize("zero_copy,pull", [(False, "kernel:256"), (False, "copy"), (True, "copy")])
def test_prefetching_local_group_matches_oracle(tmp_path, zero_copy, pull):
    """LocalGroup(prefetch=True): every granted fetch starts on the learners' side streams as
    soon as the whole round has published, so it overlaps the training step that follows
    (tools/overlap_trace.py); the trajectory stays the lock-step one."""
    rng = np.random.default_rng(19)
    G, n, T = 3, 200_003, 8
    names = ["p%d" % g for g in range(G)]
    init = rng.standard_normal((G, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    send = [[1.0 + 0.1 * g + r for g in range(G)] for r in range(T)]
    wait = [[1.5 + 0.1 * g + r for g in range(G)] for r in range(T)]
    seeds = [41 + g for g in range(G)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, 0.8, seeds)
    cfg = tmp_path / "pre.yaml"
    write_cfg(cfg, names, 0.8, "clock", 0.0, None)
    group = LocalGroup(prefetch=True, zero_copy=zero_copy)
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group, pull=pull) for g in range(G)]
    for r in range(T):
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g], reuse_snapshot=r > 0)
        for g in range(G):
            torch.cuda._sleep(200_000)                       # a "training step" behind the pulls
            flats[g].add_(torch.from_numpy(deltas[r, g]).to(DEV))
        for g in range(G):
            conns[g].update_wait_average(flats[g], wait[r][g], write_through=True)
        for g in range(G):
            assert olerp.bits_equal(flats[g].cpu().numpy(), exp["params"][r, g]), (r, g)
            assert conns[g].clock == exp["clocks"][r, g]
    for c in conns:
        c.close()


def test_resumed_gossip_continues_the_uninterrupted_one(tmp_path):
    """Gossip-state checkpoint (DpwaConnection.state_dict / load_state_dict, extension): three
    learners (clock interpolation, fetch_probability 0.7) run 12 rounds; the same learners run 6,
    are checkpointed (gossip state + parameters), closed, and new connections with other seeds
    resume from the checkpoint for 6 more.  Rounds 7-12 -- peers, clocks and parameters -- equal
    the uninterrupted run's bit for bit."""
    names = ["r0", "r1", "r2"]
    cfg = tmp_path / "resume.yaml"
    write_cfg(cfg, names, 0.7, "clock", 0.0, None)
    rng = np.random.default_rng(13)
    n, T, cut = 10_007, 12, 6
    init = rng.standard_normal((3, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, 3, n))).astype(np.float32)

    def run(conns, flats, rounds):
        rec = []
        for r in rounds:
            for c, f in zip(conns, flats):
                c.update_send(f, 1.0 + r)
            peers = []
            for c, f in zip(conns, flats):
                payload, _ = c.update_wait_average(f, 2.0 + r)
                peers.append(payload.peer if payload is not None else None)
            for g, f in enumerate(flats):
                f.add_(torch.from_numpy(deltas[r, g]).to(DEV))
            torch.cuda.synchronize()
            rec.append((peers, [c.clock for c in conns], [f.cpu().numpy().copy() for f in flats]))
        return rec

    group = LocalGroup()
    conns = [DpwaConnection(nm, str(cfg), seed=200 + g, group=group) for g, nm in enumerate(names)]
    flats = [torch.from_numpy(init[g].copy()).to(DEV) for g in range(3)]
    full = run(conns, flats, range(T))
    for c in conns:
        c.close()

    group = LocalGroup()
    conns = [DpwaConnection(nm, str(cfg), seed=200 + g, group=group) for g, nm in enumerate(names)]
    flats = [torch.from_numpy(init[g].copy()).to(DEV) for g in range(3)]
    first = run(conns, flats, range(cut))
    states = [c.state_dict() for c in conns]
    saved = [f.clone() for f in flats]
    for c in conns:
        c.close()
    group = LocalGroup()
    conns = [DpwaConnection(nm, str(cfg), seed=900 + g, group=group) for g, nm in enumerate(names)]
    for c, st in zip(conns, states):
        c.load_state_dict(st)
    second = run(conns, saved, range(cut, T))
    for c in conns:
        c.close()
    for r, (a, b) in enumerate(zip(full, first + second)):
        assert a[0] == b[0] and a[1] == b[1], (r, a[:2], b[:2])
        for g in range(3):
            assert olerp.bits_equal(a[2][g], b[2][g]), (r, g)
