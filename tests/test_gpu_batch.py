"""The batched averaging dispatch (k_lerp_batch): the averages of several co-resident learners
of one round in ONE launch (LocalGroup; pytorch.py:66-68 once per learner).  Every entry must
be exactly the single-learner fused average -- factor, clock update (dpwa.py:139-155), lerp,
write-through copy, ragged tail, ZeroDivision no-op -- against the CPU oracle, and the
connection- and adapter-level calls must follow the oracle's gossip trajectory (peers, clocks,
parameters) as the one-by-one calls do."""
import ctypes

import numpy as np
import pytest
import torch

from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter, _lib
from dpwa_amd.group import LocalGroup
from oracle import gossip as ogossip
from oracle import lerp as olerp
from oracle import policy as opolicy
from tests.test_gpu_gossip import Net
from tests.test_gpu_kernels import average_slot, from_u16, header_bytes, stream, to_u16

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
SIZES = [0, 1, 5, 4099, 65536 + 13, (1 << 20) + 5, 3, 777777]


def _entries(sizes, dtype, seed, write_through, method="clock", zero_div_at=None):
    rng = np.random.default_rng(seed)
    ents = []
    for i, n in enumerate(sizes):
        p32 = rng.standard_normal(n).astype(np.float32)
        q32 = rng.standard_normal(n).astype(np.float32)
        my_clock, peer_clock = float(i + 1), float(3 * i + 2)
        loss, peer_loss = 0.5 + 0.1 * i, 0.25 + 0.2 * i
        if zero_div_at == i:
            loss, peer_loss = 0.0, 0.0
        res = opolicy.factor_and_clock(method, None, 0.0, my_clock, peer_clock, loss, peer_loss) \
            if zero_div_at != i else None
        if dtype == "f32":
            exp = p32.copy()
            if res is not None:
                olerp.c_lerp_f32_(exp, q32, res[0])
            p, q = torch.from_numpy(p32).to(DEV), torch.from_numpy(q32).to(DEV)
        else:
            pu, qu = olerp.f32_to_bf16(p32), olerp.f32_to_bf16(q32)
            exp = pu.copy()
            if res is not None:
                olerp.c_lerp_bf16_(exp, qu, res[0])
            p, q = from_u16(pu), from_u16(qu)
        ents.append(dict(n=n, p=p, slot=average_slot(q, peer_clock, peer_loss), exp=exp, res=res,
                         my_clock=my_clock, loss=loss,
                         snap=torch.full_like(p, float("nan")) if write_through else None,
                         clock=torch.tensor([my_clock, -1.0], dtype=torch.float64, device=DEV),
                         coef=torch.zeros(32, dtype=torch.uint8, device=DEV)))
    return ents


def _descs(ents):
    d = (_lib.AverageDesc * len(ents))()
    for j, e in enumerate(ents):
        d[j] = _lib.AverageDesc(e["p"].data_ptr(), e["slot"].data_ptr(), e["n"], e["clock"].data_ptr(), e["loss"],
                                e["coef"].data_ptr(), e["snap"].data_ptr() if e["snap"] is not None else None)
    return d


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("write_through", [False, True])
@pytest.mark.parametrize("count", [1, 2, 3, 8])
def test_average_many_entry_point_vs_oracle(dtype, write_through, count):
    """dpwa_average_many over ragged sizes (0, 1, odd tails, > 1M): each entry bit-exact with
    the C oracle lerp under its own clock-interpolation factor; each entry's clock and
    coefficient block written; write-through copies equal the averaged parameters."""
    sizes = SIZES[:count]
    ents = _entries(sizes, dtype, 50 + count, write_through)
    cfg = _lib.Interp(_lib.INTERP_CLOCK, 0, 0.0, 0.0)
    _lib.call("dpwa_average_many", _lib.F32 if dtype == "f32" else _lib.BF16, _descs(ents), len(ents),
              ctypes.byref(cfg), stream(), None, None)
    torch.cuda.synchronize()
    for i, e in enumerate(ents):
        got = e["p"].cpu().numpy() if dtype == "f32" else to_u16(e["p"])
        assert olerp.bits_equal(got, e["exp"]), (i, e["n"])
        c = _lib.Coef.from_buffer_copy(e["coef"].cpu().numpy().tobytes())
        assert c.status == 0 and c.factor == e["res"][0], i
        assert e["clock"][1].item() == e["res"][1], i          # dpwa.py:150
        if write_through and e["n"]:
            assert torch.equal(e["snap"].view(torch.uint8), e["p"].view(torch.uint8)), i


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_average_many_zero_division_entry_is_a_noop(dtype):
    """Loss interpolation with loss + peer_loss == 0 in one entry (the reference's
    ZeroDivisionError, interpolation.py:31-33): that entry keeps its parameters and clock and
    still writes its snapshot; the other entries of the same dispatch average normally."""
    ents = _entries([4099, 65536 + 13, 5], dtype, 7, True, method="loss", zero_div_at=1)
    before = ents[1]["p"].clone()
    cfg = _lib.Interp(_lib.INTERP_LOSS, 0, 0.0, 0.0)
    _lib.call("dpwa_average_many", _lib.F32 if dtype == "f32" else _lib.BF16, _descs(ents), len(ents),
              ctypes.byref(cfg), stream(), None, None)
    torch.cuda.synchronize()
    c1 = _lib.Coef.from_buffer_copy(ents[1]["coef"].cpu().numpy().tobytes())
    assert c1.status == _lib.STATUS_ZERO_DIVISION
    assert torch.equal(ents[1]["p"], before) and torch.equal(ents[1]["snap"], before)
    assert ents[1]["clock"][1].item() == ents[1]["my_clock"]
    for i in (0, 2):
        got = ents[i]["p"].cpu().numpy() if dtype == "f32" else to_u16(ents[i]["p"])
        assert olerp.bits_equal(got, ents[i]["exp"]), i


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("write_through", [False, True])
@pytest.mark.parametrize("n", [0, 1, 5, 4099, 8 * 64 * 4, 65536 + 13, (1 << 20) + 5])
@pytest.mark.parametrize("zero_div_at", [None, 0, 1])
def test_two_equal_entries_vs_oracle(dtype, write_through, n, zero_div_at):
    """Two equal-size in-place entries -- the N=1 reference loop's write-through pair, its spans
    dealt round-robin: each bit-exact with the C oracle at ragged sizes, clocks and coefficient
    blocks written, a ZeroDivision entry (loss interpolation, loss + peer loss == 0) left unchanged
    with its snapshot still written, whichever of the two it is."""
    method = "loss" if zero_div_at is not None else "clock"
    ents = _entries([n, n], dtype, 90 + n % 97, write_through, method=method, zero_div_at=zero_div_at)
    before = [e["p"].clone() for e in ents]
    cfg = _lib.Interp(_lib.INTERP_LOSS if method == "loss" else _lib.INTERP_CLOCK, 0, 0.0, 0.0)
    _lib.call("dpwa_average_many", _lib.F32 if dtype == "f32" else _lib.BF16, _descs(ents), 2,
              ctypes.byref(cfg), stream(), None, None)
    torch.cuda.synchronize()
    for i, e in enumerate(ents):
        c = _lib.Coef.from_buffer_copy(e["coef"].cpu().numpy().tobytes())
        if i == zero_div_at:
            assert c.status == _lib.STATUS_ZERO_DIVISION and torch.equal(e["p"], before[i])
            assert e["clock"][1].item() == e["my_clock"]
        else:
            got = e["p"].cpu().numpy() if dtype == "f32" else to_u16(e["p"])
            assert olerp.bits_equal(got, e["exp"]), (i, n)
            assert c.status == 0 and c.factor == e["res"][0] and e["clock"][1].item() == e["res"][1], i
        if write_through and n:
            assert torch.equal(e["snap"].view(torch.uint8), e["p"].view(torch.uint8)), i


def test_average_many_argument_errors():
    ents = _entries([64, 64], "f32", 3, True)
    d = _descs(ents)
    cfg = _lib.Interp(_lib.INTERP_CLOCK, 0, 0.0, 0.0)
    lib = _lib.load()
    assert lib.dpwa_average_many(_lib.F32, d, 0, ctypes.byref(cfg), stream(), None, None) == _lib.ERR_ARG
    assert lib.dpwa_average_many(_lib.F32, d, 9, ctypes.byref(cfg), stream(), None, None) == _lib.ERR_ARG
    d[1].snap_payload = None                                     # mixed write-through
    assert lib.dpwa_average_many(_lib.F32, d, 2, ctypes.byref(cfg), stream(), None, None) == _lib.ERR_ARG
    d[1].snap_payload = ents[1]["snap"].data_ptr()
    d[0].param = ents[0]["p"].data_ptr() + 4                     # unaligned
    assert lib.dpwa_average_many(_lib.F32, d, 2, ctypes.byref(cfg), stream(), None, None) == _lib.ERR_ARG
    torch.cuda.synchronize()


def _write_cfg(path, names, fp, interp):
    lines = ["- nodes:"] + ["  - {name: %s, host: localhost, port: %d}" % (n, 46000 + i) for i, n in enumerate(names)]
    lines += ["- fetch_probability: %r" % fp, "- timeout_ms: 2500", "- interpolation: %s" % interp,
              "- divergence_threshold: 0", "- constant: { value: 0.5 }", "- clock: 0", "- loss: 0"]
    path.write_text("\n".join(lines) + "\n")


@pytest.mark.parametrize("write_through", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_update_wait_average_many_matches_oracle(tmp_path, write_through, dtype):
    """Four co-resident learners, clock interpolation, fetch_probability 0.7 (some rounds have
    no fetch), 12 rounds: every round's averages through ONE update_wait_average_many call;
    parameters, clocks and peers bit-exact with oracle/gossip.py, and equal to the same rounds
    run one learner at a time."""
    G, n, T, fp = 4, 40_009, 12, 0.7
    names = ["b%d" % g for g in range(G)]
    cfg = tmp_path / "batch.yaml"
    _write_cfg(cfg, names, fp, "clock")
    rng = np.random.default_rng(11)
    init32 = rng.standard_normal((G, n)).astype(np.float32)
    d32 = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    send = [[1.0 + 0.1 * g + r for g in range(G)] for r in range(T)]
    wait = [[0.9 + 0.1 * g + r for g in range(G)] for r in range(T)]
    seeds = [300 + g for g in range(G)]
    if dtype == torch.float32:
        init, deltas = init32, d32
        exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, fp, seeds)
        to_dev = lambda a: torch.from_numpy(a).to(DEV)               # noqa: E731
        to_np = lambda t: t.cpu().numpy()                            # noqa: E731
    else:
        init, deltas = olerp.f32_to_bf16(init32), olerp.f32_to_bf16(d32)
        exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, fp, seeds,
                               lerp=olerp.lerp_bf16, add=ogossip.add_bf16)
        to_dev = from_u16
        to_np = to_u16
    runs = {}
    for mode in ("batched", "single"):
        group = LocalGroup()
        conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
        flats = [to_dev(init[g]) for g in range(G)]
        peers = []
        for r in range(T):
            for g in range(G):
                conns[g].update_send(flats[g], send[r][g], reuse_snapshot=write_through and r > 0)
            for g in range(G):
                flats[g].add_(to_dev(deltas[r, g]))
            if mode == "batched":
                res = DpwaConnection.update_wait_average_many(conns, flats, wait[r], write_through=write_through)
            else:
                res = [conns[g].update_wait_average(flats[g], wait[r][g], write_through=write_through)
                       for g in range(G)]
            peers.append([p.peer if p is not None else "" for p, _ in res])
            for g in range(G):
                assert conns[g].clock == exp["clocks"][r, g], (mode, r, g)
                assert olerp.bits_equal(to_np(flats[g]), exp["params"][r, g]), (mode, r, g)
        runs[mode] = peers
        for g in range(G):
            want = [(exp["picks"][r][g][-1] if exp["picks"][r][g] else "") for r in range(T)]
            assert [peers[r][g] for r in range(T)] == want, (mode, g)
            conns[g].close()
    assert runs["batched"] == runs["single"]


def test_adapter_update_wait_many_matches_one_by_one(tmp_path):
    """DpwaPyTorchAdapter.update_wait_many over three models on one GPU gives exactly the
    parameters and clocks of calling update_wait on each (write-through default, so the next
    update_send reuses the batched dispatch's snapshots)."""
    shapes = [(64, 3, 3, 3), (64,), (10, 64), (10,), (7, 5)]
    names = ["a0", "a1", "a2"]
    cfg = tmp_path / "ad.yaml"
    _write_cfg(cfg, names, 1.0, "clock")
    results = {}
    for mode in ("many", "single"):
        torch.manual_seed(5)
        nets = [Net(shapes).to(DEV) for _ in names]
        grp = LocalGroup()
        ads = [DpwaPyTorchAdapter(nets[g], names[g], str(cfg), seed=40 + g, group=grp) for g in range(3)]
        for r in range(6):
            for g, ad in enumerate(ads):
                ad.update_send(1.0 + g + r)
            with torch.no_grad():
                for net in nets:
                    for p in net.parameters():
                        p.add_(0.01)
            if mode == "many":
                DpwaPyTorchAdapter.update_wait_many(ads, [0.5 + g + r for g in range(3)])
            else:
                for g, ad in enumerate(ads):
                    ad.update_wait(0.5 + g + r)
        results[mode] = ([torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu() for net in nets],
                         [ad.connection.clock for ad in ads])
        for ad in ads:
            ad.connection.close()
    for a, b in zip(results["many"][0], results["single"][0]):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    assert results["many"][1] == results["single"][1]


def test_wire_write_through_serves_the_update_send_loss(tmp_path):
    """A WireConnection averaging write-through with a float32 loss tensor (advisor items on
    bridge._loss and the write-ahead header): the factor reads the float32 loss correctly (loss
    interpolation against the oracle) and the snapshot served after a header-only publish
    carries the loss given to that update_send, not a placeholder."""
    from dpwa_amd.bridge import SnapshotCodec, WireConnection
    from tests.test_gpu_bridge import free_port, wire_cfg
    G, n, T = 2, 5_003, 4
    names = ["u0", "u1"]
    ports = [free_port() for _ in range(G)]
    cfg = tmp_path / "wt.yaml"
    wire_cfg(cfg, names, ports, fp=1.0, interp="loss")
    rng = np.random.default_rng(21)
    init = rng.standard_normal((G, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    send = [[float(np.float32(1.5 + 0.25 * g + 0.1 * r)) for g in range(G)] for r in range(T)]
    wait = [[float(np.float32(1.25 + 0.5 * g + 0.1 * r)) for g in range(G)] for r in range(T)]
    seeds = [90, 91]
    exp = ogossip.simulate(names, init, deltas, send, wait, "loss", None, 0.0, 1.0, seeds)
    conns = [WireConnection(names[g], str(cfg), codec=SnapshotCodec.single("w", n), seed=seeds[g], eager=False)
             for g in range(G)]
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    for r in range(T):
        for g in range(G):
            conns[g].update_send(flats[g], torch.tensor(send[r][g], dtype=torch.float32, device=DEV),
                                 reuse_snapshot=r > 0)
        torch.cuda.synchronize()
        for g in range(G):
            state, _, release = conns[g]._snapshot()
            release()
            assert state["loss"] == send[r][g], (r, g, state)
        for g in range(G):
            flats[g].add_(torch.from_numpy(deltas[r, g]).to(DEV))
        for g in range(G):
            conns[g].update_wait_average(flats[g], torch.tensor(wait[r][g], dtype=torch.float32, device=DEV),
                                         write_through=True)
        torch.cuda.synchronize()
    for g in range(G):
        assert olerp.bits_equal(flats[g].cpu().numpy(), exp["params"][-1, g]), g
        assert conns[g].clock == exp["clocks"][-1, g]
        conns[g].close()


def test_average_many_beyond_4gib_offsets():
    """Two bf16 entries of 2^31 + 1001 elements (4.3 GB per operand: byte offsets past 2^32) in one
    batched write-through dispatch: sampled windows at the start, around 2^30 and 2^31 elements
    and at the ragged end of both entries, against the oracle bf16 lerp of the same windows."""
    n = (1 << 31) + 1001
    cfg = _lib.Interp(_lib.INTERP_CLOCK, 0, 0.0, 0.0)
    hdr = _lib.SLOT_PAYLOAD_OFFSET // 2
    ents = []
    for i in range(2):
        g = torch.Generator(device=DEV).manual_seed(70 + i)
        p = torch.empty(n, dtype=torch.bfloat16, device=DEV).normal_(generator=g)
        slot = torch.zeros(hdr + n, dtype=torch.bfloat16, device=DEV)
        slot[hdr:].normal_(generator=g)
        slot.view(torch.uint8)[:256].copy_(torch.frombuffer(bytearray(header_bytes(3.0 + i, 1.0)), dtype=torch.uint8))
        snap = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        clock = torch.tensor([1.0 + i, -1.0], dtype=torch.float64, device=DEV)
        coef = torch.zeros(32, dtype=torch.uint8, device=DEV)
        ents.append(dict(p=p, slot=slot, snap=snap, clock=clock, coef=coef, my=1.0 + i, peer=3.0 + i))
    wins = [0, (1 << 30) - 5, (1 << 31) - 7, n - 4096]
    before = [[to_u16(e["p"][w:w + 4096]) for w in wins] for e in ents]
    peers = [[to_u16(e["slot"][hdr + w:hdr + w + 4096]) for w in wins] for e in ents]
    d = (_lib.AverageDesc * 2)()
    for j, e in enumerate(ents):
        d[j] = _lib.AverageDesc(e["p"].data_ptr(), e["slot"].data_ptr(), n, e["clock"].data_ptr(), 1.0,
                                e["coef"].data_ptr(), e["snap"].data_ptr())
    _lib.call("dpwa_average_many", _lib.BF16, d, 2, ctypes.byref(cfg), stream(), None, None)
    torch.cuda.synchronize()
    for j, e in enumerate(ents):
        f, new_clock = opolicy.factor_and_clock("clock", None, 0.0, e["my"], e["peer"], 1.0, 1.0)
        assert e["clock"][1].item() == new_clock
        for k, w in enumerate(wins):
            want = olerp.lerp_bf16(before[j][k], peers[j][k], f)
            assert olerp.bits_equal(to_u16(e["p"][w:w + 4096]), want), (j, w)
            assert olerp.bits_equal(to_u16(e["snap"][w:w + 4096]), want), (j, w)
    del ents
    torch.cuda.empty_cache()


def test_update_wait_average_many_unaligned_buffers_fall_back(tmp_path):
    """Flat buffers that are not 16-B aligned (views at a 4-byte offset) cannot join the batched
    dispatch: each such average is launched on its own (the element-wise kernel), with the same
    results as the single calls -- checked against oracle/gossip.py."""
    G, n, T = 3, 10_007, 5
    names = ["u%d" % g for g in range(G)]
    cfg = tmp_path / "ua.yaml"
    _write_cfg(cfg, names, 1.0, "clock")
    rng = np.random.default_rng(12)
    init = rng.standard_normal((G, n)).astype(np.float32)
    deltas = (0.01 * rng.standard_normal((T, G, n))).astype(np.float32)
    send = [[1.0 + g + r for g in range(G)] for r in range(T)]
    wait = [[1.5 + g + r for g in range(G)] for r in range(T)]
    seeds = [500 + g for g in range(G)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, 1.0, seeds)
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
    backing = [torch.zeros(n + 1, device=DEV) for _ in range(G)]
    flats = [b[1:] for b in backing]                       # 4-byte offset: not 16-B aligned
    for g in range(G):
        flats[g].copy_(torch.from_numpy(init[g]).to(DEV))
    for r in range(T):
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g], reuse_snapshot=r > 0)
        for g in range(G):
            flats[g].add_(torch.from_numpy(deltas[r, g]).to(DEV))
        DpwaConnection.update_wait_average_many(conns, flats, wait[r], write_through=True)
        for g in range(G):
            assert olerp.bits_equal(flats[g].cpu().numpy(), exp["params"][r, g]), (r, g)
            assert conns[g].clock == exp["clocks"][r, g]
    for c in conns:
        c.close()
