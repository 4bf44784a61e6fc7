"""configs[1]'s self-peer on one GPU: a learner whose YAML lists a second node entry at its own
host:port averages with the snapshot it published itself -- the reference's TxThread dials that
address and reaches its own RxThread (conn.py:246-251 -> 98-110).  `LocalGroup` resolves the
entry by address to the learner itself and the average reads its own published slot in place.

* the reference's own self-peer trajectories (tests/golden/gossip_self.*, make_golden.py
  gen_gossip_self: constant / clock / loss interpolation, fetch_probability 1 and 0.7) replayed
  bit for bit through the adapter's default (write-through), the connection's write-through
  rounds and the split update_wait + average;
* configs[1] at its full size (11,173,962 fp32, constant 0.5, fetch_probability 1) in the
  reference loop order with a training step between update_send and update_wait, every round's
  whole vector against the C oracle (the bench's headline workload)."""
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
RESNET18_NUMEL = 11_173_962


class Net(torch.nn.Module):
    def __init__(self, shapes):
        super().__init__()
        for i, s in enumerate(shapes):
            self.register_parameter("p%d" % i, torch.nn.Parameter(torch.zeros(s)))


def write_self_cfg(path, fp, interp, thr, value, port=48100):
    """The reference's YAML with the learner and a second entry at the learner's own address."""
    lines = ["- nodes:", "  - {name: w1, host: localhost, port: %d}" % port,
             "  - {name: w1-self, host: localhost, port: %d}" % port,
             "- fetch_probability: %r" % fp, "- timeout_ms: 2500", "- interpolation: %s" % interp,
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


def step(net, delta):
    with torch.no_grad():
        off = 0
        for _, p in net.named_parameters():
            k = p.numel()
            p.data.add_(torch.from_numpy(delta[off:off + k]).to(DEV).view(p.shape))
            off += k


@pytest.mark.parametrize("form", ["adapter", "connection-wt", "split"])
def test_self_peer_matches_reference_trajectories(tmp_path, form):
    meta = load_json("gossip_self.json")
    z = load_npz("gossip_self.npz")
    shapes = [tuple(s) for s in meta["shapes"]]
    for case in meta["cases"]:
        k = case["key"]
        cfg = tmp_path / ("%s_%s.yaml" % (k, form))
        write_self_cfg(cfg, case["fetch_probability"], case["interpolation"], case["divergence_threshold"],
                       case["value"])
        init, deltas = z[k + "_init"], z[k + "_deltas"]
        group = LocalGroup()
        if form == "adapter":
            net = Net(shapes).to(DEV)
            load_flat(net, init[0])
            ad = DpwaPyTorchAdapter(net, "w1", str(cfg), seed=case["seeds"][0], group=group)
            conn = ad.connection
        else:
            conn = DpwaConnection("w1", str(cfg), seed=case["seeds"][0], group=group)
            flat = torch.from_numpy(init[0].copy()).to(DEV)
        assert [p.name for p in conn.peers] == ["w1-self"]
        wt_prev = False
        for r in range(deltas.shape[0]):  # noqa: B007
            if form == "adapter":
                ad.update_send(case["send_loss"][r][0])
                step(net, deltas[r, 0])
                ad.update_wait(case["wait_loss"][r][0])
                got = flat_params(net)
            else:
                conn.update_send(flat, case["send_loss"][r][0], reuse_snapshot=wt_prev)
                flat.add_(torch.from_numpy(deltas[r, 0]).to(DEV))
                if form == "split":
                    payload, _ = conn.update_wait(case["wait_loss"][r][0])
                    if payload is not None:
                        conn.average(flat)
                    wt_prev = False
                else:
                    # the reference order: the step comes after update_send, so nothing writes the
                    # parameters between this average and the next update_send -- its snapshot is
                    # what this average writes through (a round without an average publishes in full)
                    payload, _ = conn.update_wait_average(flat, case["wait_loss"][r][0], write_through=True)
                    wt_prev = payload is not None
                got = flat.cpu().numpy()
            fetched = bool(z[k + "_fetching"][r, 0])
            assert conn.fetching is False
            assert ([conn.last_fetch_peer] if fetched and conn.last_fetch_peer else []) == case["picks"][r][0], (k, r)
            assert conn.clock == z[k + "_clocks"][r, 0], (k, r)
            if fetched:
                assert float(conn._learner.read_coef().factor) == z[k + "_factors"][r, 0], (k, r)
            assert olerp.bits_equal(got, z[k + "_params"][r, 0]), (form, k, r)
        conn.close()


def test_self_peer_write_through_rounds_match_oracle(tmp_path):
    """The bench's round: update_send(reuse_snapshot) -> update_wait_average(write_through), no step
    in between (the snapshot is then exactly what the last average wrote through), 12 rounds with
    clock interpolation and fetch_probability 0.7 (rounds without an average publish in full) --
    against oracle/gossip.py with the self-peer node list."""
    rng = np.random.default_rng(41)
    n, T = 100_003, 12
    init = rng.standard_normal((1, n)).astype(np.float32)
    deltas = np.zeros((T, 1, n), np.float32)
    send = [[1.0 + 0.1 * r] for r in range(T)]
    wait = [[0.9 + 0.1 * r] for r in range(T)]
    exp = ogossip.simulate(["w1"], init, deltas, send, wait, "clock", None, 0.0, 0.7, [17],
                           nodes=["w1", "w1-self"], serves={"w1-self": 0})
    cfg = tmp_path / "wt.yaml"
    write_self_cfg(cfg, 0.7, "clock", 0.0, None)
    conn = DpwaConnection("w1", str(cfg), seed=17, group=LocalGroup())
    flat = torch.from_numpy(init[0].copy()).to(DEV)
    reuse = False
    for r in range(T):
        conn.update_send(flat, send[r][0], reuse_snapshot=reuse)
        payload, _ = conn.update_wait_average(flat, wait[r][0], write_through=True)
        reuse = payload is not None
        assert conn.clock == exp["clocks"][r, 0], r
        assert olerp.bits_equal(flat.cpu().numpy(), exp["params"][r, 0]), r
    conn.close()


def test_configs1_self_peer_full_size_reference_order(tmp_path):
    """configs[1] as the bench's headline runs it: one learner of 11,173,962 fp32, its peer its own
    snapshot, constant 0.5, fetch_probability 1, the reference loop order (update_send, a training
    step writing every parameter, update_wait with the write-through average).  Every round's whole
    vector equals the C oracle's lerp of the pre-step snapshot into the stepped parameters."""
    n = RESNET18_NUMEL
    cfg = tmp_path / "c1.yaml"
    write_self_cfg(cfg, 1.0, "constant", 0.0, 0.5)
    g = torch.Generator(device=DEV).manual_seed(0)
    flat = torch.randn(n, device=DEV, generator=g)
    upd = (1e-3 * torch.randn(n, device=DEV, generator=g))
    conn = DpwaConnection("w1", str(cfg), seed=1000, group=LocalGroup())
    host = flat.cpu().numpy()
    u = upd.cpu().numpy()
    reuse = False
    for r in range(6):
        conn.update_send(flat, 1.0, reuse_snapshot=reuse)
        snap = host.copy()
        flat.sub_(upd)                              # the step (after the snapshot was taken)
        host = (host - u).astype(np.float32)
        payload, _ = conn.update_wait_average(flat, 1.0, write_through=True)
        assert payload is not None and payload.peer == "w1-self"
        olerp.c_lerp_f32_(host, snap, 0.5)
        assert olerp.bits_equal(flat.cpu().numpy(), host), r
        # nothing writes the parameters between update_wait and the next update_send (the step
        # comes after update_send): the next publish reuses the snapshot the average wrote through
        reuse = True
    # a write between update_wait and update_send: the caller publishes in full
    flat.sub_(upd)
    host = (host - u).astype(np.float32)
    conn.update_send(flat, 1.0, reuse_snapshot=False)
    snap = host.copy()
    conn.update_wait_average(flat, 1.0, write_through=True)
    olerp.c_lerp_f32_(host, snap, 0.5)
    assert olerp.bits_equal(flat.cpu().numpy(), host)
    conn.close()


@pytest.mark.parametrize("form", ["bf16-write-through", "f32-resident", "bf16-resident"])
def test_self_peer_other_forms_match_oracle(tmp_path, form):
    """The self-peer in bf16 (torch-eager two-rounding lerp) with write-through rounds in the
    reference order, and with resident parameters (the published slot is both the parameters and
    the peer; the step after update_wait, as a resident loop runs) -- 12 rounds, clock
    interpolation, fetch_probability 0.7 (rounds without an average publish in full / relocate),
    ragged size, against oracle/gossip.py with the self-peer node list."""
    from tests.test_gpu_kernels import from_u16, to_u16
    bf16 = form.startswith("bf16")
    resident = form.endswith("resident")
    rng = np.random.default_rng(43)
    n, T = 100_003, 12
    init32 = rng.standard_normal((1, n)).astype(np.float32)
    d32 = (0.01 * rng.standard_normal((T, 1, n))).astype(np.float32)
    if bf16:
        init, deltas = olerp.f32_to_bf16(init32), olerp.f32_to_bf16(d32)
        to_dev, to_host, kw = from_u16, to_u16, dict(lerp=olerp.lerp_bf16, add=ogossip.add_bf16)
    else:
        init, deltas = init32, d32
        to_dev, to_host, kw = (lambda a: torch.from_numpy(a).to(DEV)), (lambda t: t.cpu().numpy()), {}
    send = [[1.0 + 0.1 * r] for r in range(T)]
    wait = [[0.9 + 0.1 * r] for r in range(T)]
    exp = ogossip.simulate(["w1"], init, deltas, send, wait, "clock", None, 0.0, 0.7, [19], train_after_wait=resident,
                           nodes=["w1", "w1-self"], serves={"w1-self": 0}, **kw)
    cfg = tmp_path / ("%s.yaml" % form)
    write_self_cfg(cfg, 0.7, "clock", 0.0, None)
    conn = DpwaConnection("w1", str(cfg), seed=19, group=LocalGroup())
    flat = to_dev(init[0].copy())
    if resident:
        conn.make_resident(flat)
        for r in range(T):
            conn.update_send(conn.parameters, send[r][0])
            conn.update_wait_average(conn.parameters, wait[r][0])
            assert conn.clock == exp["clocks"][r, 0], r
            assert np.array_equal(to_host(conn.parameters).view(np.uint32 if not bf16 else np.uint16),
                                  exp["params"][r, 0].view(np.uint32 if not bf16 else np.uint16)), r
            conn.parameters.add_(to_dev(deltas[r, 0]))                  # the step, after update_wait
    else:
        reuse = False
        for r in range(T):
            conn.update_send(flat, send[r][0], reuse_snapshot=reuse)
            flat.add_(to_dev(deltas[r, 0]))                             # the step, between the two
            payload, _ = conn.update_wait_average(flat, wait[r][0], write_through=True)
            reuse = payload is not None
            assert conn.clock == exp["clocks"][r, 0], r
            assert np.array_equal(to_host(flat).view(np.uint16), exp["params"][r, 0].view(np.uint16)), r
    conn.close()
