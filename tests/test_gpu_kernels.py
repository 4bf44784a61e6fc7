"""GPU parity of the HIP kernels (called through the C ABI) against the CPU oracle, the
reference-generated fixtures and, at full sizes, torch-eager on the same device.

Bar: bit-exact for fp32 (NaN payloads excepted) and for the bf16 two-rounding form.
"""
import ctypes
import struct

import numpy as np
import pytest
import torch

from dpwa_amd import _lib
from oracle import lerp as olerp
from oracle import policy as opolicy
from tests.helpers import hexf, load_json, load_npz, num

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return _lib.stream_handle(None)


def host_lerp(param, peer, factor):
    fn = "dpwa_lerp_f32_host" if param.dtype == torch.float32 else "dpwa_lerp_bf16_host"
    _lib.call(fn, ptr(param), ptr(peer), param.numel(), float(factor), stream())


def coef_block(factor):
    """A dpwa_coef in device memory produced by the factor kernel (constant method)."""
    clock = torch.zeros(1, dtype=torch.float64, device=DEV)
    hdr = torch.zeros(256, dtype=torch.uint8, device=DEV)
    coef = torch.zeros(32, dtype=torch.uint8, device=DEV)
    cfg = _lib.Interp(_lib.INTERP_CONSTANT, 0, float(factor), 0.0)
    _lib.call("dpwa_factor", ctypes.byref(cfg), ptr(clock), ptr(hdr), 1.0, None, ptr(coef), stream())
    return coef


def dev_lerp(param, peer, coef):
    fn = "dpwa_lerp_f32" if param.dtype == torch.float32 else "dpwa_lerp_bf16"
    _lib.call(fn, ptr(param), ptr(peer), param.numel(), ptr(coef), stream())


def to_u16(t):
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def from_u16(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).to(DEV)


def test_lerp_f32_matches_reference_fixture():
    z = load_npz("lerp_f32.npz")
    peer = torch.from_numpy(z["peer"]).to(DEV)
    for f, out in zip(z["factors"], z["out"]):
        for mode in ("host", "device"):
            p = torch.from_numpy(z["param"]).to(DEV)
            if mode == "host":
                host_lerp(p, peer, f)
            else:
                dev_lerp(p, peer, coef_block(f))
            torch.cuda.synchronize()
            assert olerp.bits_equal(p.cpu().numpy(), out), (f, mode)


def test_lerp_bf16_matches_torch_eager_fixture():
    z = load_npz("lerp_bf16.npz")
    peer = from_u16(z["peer"])
    for f, out in zip(z["factors"], z["out"]):
        p = from_u16(z["param"])
        dev_lerp(p, peer, coef_block(f))
        torch.cuda.synchronize()
        assert olerp.bits_equal(to_u16(p), out), f


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 7, 8, 9, 255, 1023, 4099, 65536 + 13, (1 << 20) + 5, 3_000_001])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_lerp_ragged_sizes_vs_c_oracle(n, dtype):
    rng = np.random.default_rng(n)
    f = float(rng.uniform())
    p32 = rng.standard_normal(n).astype(np.float32)
    q32 = rng.standard_normal(n).astype(np.float32)
    if dtype == "f32":
        exp = p32.copy()
        olerp.c_lerp_f32_(exp, q32, f)
        p, q = torch.from_numpy(p32).to(DEV), torch.from_numpy(q32).to(DEV)
        host_lerp(p, q, f)
        torch.cuda.synchronize()
        assert olerp.bits_equal(p.cpu().numpy(), exp)
    else:
        pu, qu = olerp.f32_to_bf16(p32), olerp.f32_to_bf16(q32)
        exp = pu.copy()
        olerp.c_lerp_bf16_(exp, qu, f)
        p, q = from_u16(pu), from_u16(qu)
        host_lerp(p, q, f)
        torch.cuda.synchronize()
        assert olerp.bits_equal(to_u16(p), exp)


@pytest.mark.parametrize("off_p,off_q", [(1, 0), (0, 3), (2, 2), (1, 2)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_lerp_unaligned_views(off_p, off_q, dtype):
    n = 10007
    g = torch.Generator(device="cpu").manual_seed(off_p * 10 + off_q)
    base_p = torch.randn(n + 8, generator=g).to(dtype).to(DEV)
    base_q = torch.randn(n + 8, generator=g).to(dtype).to(DEV)
    p, q = base_p[off_p:off_p + n], base_q[off_q:off_q + n]
    f = 0.3
    want = (f * q + (1 - f) * p)          # torch eager on the same device
    before_p = base_p.clone()
    host_lerp(p, q, f)
    torch.cuda.synchronize()
    assert torch.equal(p.view(torch.int16 if dtype == torch.bfloat16 else torch.int32),
                       want.view(torch.int16 if dtype == torch.bfloat16 else torch.int32))
    # nothing outside the view was touched
    assert torch.equal(base_p[:off_p], before_p[:off_p])
    assert torch.equal(base_p[off_p + n:], before_p[off_p + n:])


@pytest.mark.parametrize("n,dtype", [(100_000_000, torch.float32), (1_000_000_000, torch.bfloat16)])
def test_lerp_full_size_vs_torch_eager(n, dtype):
    """BASELINE configs 3/4 sizes: bit-equal to torch-eager `f*t + (1-f)*p` on the device,
    plus size-independent properties (f=0 identity, f=1 -> peer, symmetry at f=0.5)."""
    g = torch.Generator(device=DEV).manual_seed(1)
    p = torch.randn(n, device=DEV, generator=g, dtype=torch.float32).to(dtype)
    q = torch.randn(n, device=DEV, generator=g, dtype=torch.float32).to(dtype)
    iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
    for f in (1.0 / 3.0, 0.5):
        want = f * q + (1 - f) * p
        got = p.clone()
        host_lerp(got, q, f)
        assert torch.equal(got.view(iv), want.view(iv)), f
        del want, got
    sym_a, sym_b = p.clone(), q.clone()
    host_lerp(sym_a, q, 0.5)
    host_lerp(sym_b, p, 0.5)
    assert torch.equal(sym_a.view(iv), sym_b.view(iv))
    del sym_a, sym_b
    ident = p.clone()
    host_lerp(ident, q, 0.0)
    assert torch.equal(ident.view(iv), p.view(iv))
    host_lerp(ident, q, 1.0)
    assert torch.equal(ident.view(iv), q.view(iv))
    torch.cuda.synchronize()


def header_bytes(clock, loss):
    return struct.pack("<ddQqii", clock, loss, 1, 0, 0, 0) + bytes(216)


def test_factor_kernel_matches_reference_policy_traces():
    """Every averaging round of tests/golden/policy.json recomputed by the device factor kernel."""
    data = load_json("policy.json")
    clock = torch.zeros(1, dtype=torch.float64, device=DEV)
    coef = torch.zeros(32, dtype=torch.uint8, device=DEV)
    hdr = torch.zeros(256, dtype=torch.uint8, device=DEV)
    loss_dev = torch.zeros(1, dtype=torch.float64, device=DEV)
    checked = raised = 0
    for case in data["cases"]:
        cfg = _lib.Interp(opolicy.METHODS[case["interpolation"]], 0, float(case["value"] or 0.0),
                          float(case["divergence_threshold"]))
        L = opolicy.OracleLearner("w2", ["w1", "w3"], case["fetch_probability"], case["interpolation"],
                                  case["value"], case["divergence_threshold"], case["seed"])
        for r in case["rounds"]:
            L.update_send(num(r["send_loss"]))
            if not (r["fetching"] and r["has_payload"]):
                if r["fetching"]:
                    L.update_wait(0.0, None, False)
                continue
            clock.fill_(float(L.clock))
            hdr.copy_(torch.frombuffer(bytearray(header_bytes(float(num(r["peer_clock"])),
                                                              float(num(r["peer_loss"])))), dtype=torch.uint8))
            wl = float(num(r["wait_loss"]))
            use_dev = (checked % 2) == 1
            loss_dev.fill_(wl)
            _lib.call("dpwa_factor", ctypes.byref(cfg), ptr(clock), ptr(hdr), 0.0 if use_dev else wl,
                      ptr(loss_dev) if use_dev else None, ptr(coef), stream())
            c = _lib.Coef.from_buffer_copy(coef.cpu().numpy().tobytes())
            new_clock = clock.item()
            if r["raises"]:
                assert c.status == _lib.STATUS_ZERO_DIVISION
                assert new_clock == float(L.clock)
                L.fetching = False
                raised += 1
                continue
            L.update_wait(wl, {"clock": num(r["peer_clock"]), "loss": num(r["peer_loss"])}, True)
            assert c.status == 0
            assert c.factor == hexf(r["factor_hex"])
            assert new_clock == hexf(r["clock_hex"]) == c.new_clock
            assert c.a == np.float32(c.factor) and c.b == np.float32(1.0 - c.factor)
            checked += 1
    assert checked > 500 and raised > 5


def test_zero_division_status_makes_lerp_a_noop():
    clock = torch.zeros(1, dtype=torch.float64, device=DEV)
    hdr = torch.zeros(256, dtype=torch.uint8, device=DEV)
    coef = torch.zeros(32, dtype=torch.uint8, device=DEV)
    cfg = _lib.Interp(_lib.INTERP_LOSS, 0, 0.0, 0.0)
    _lib.call("dpwa_factor", ctypes.byref(cfg), ptr(clock), ptr(hdr), 0.0, None, ptr(coef), stream())
    p = torch.randn(1000, device=DEV)
    q = torch.randn(1000, device=DEV)
    before = p.clone()
    dev_lerp(p, q, coef)
    torch.cuda.synchronize()
    assert torch.equal(p, before)


def average_slot(peer_payload, peer_clock, peer_loss):
    """A peer snapshot laid out as a learner's slot (ABI 3): dpwa_header at 0, payload at
    DPWA_SLOT_PAYLOAD_OFFSET."""
    off = _lib.SLOT_PAYLOAD_OFFSET
    raw = torch.zeros(off + peer_payload.numel() * peer_payload.element_size(), dtype=torch.uint8, device=DEV)
    raw[:256].copy_(torch.frombuffer(bytearray(header_bytes(peer_clock, peer_loss)), dtype=torch.uint8))
    if peer_payload.numel():
        raw[off:].copy_(peer_payload.view(torch.uint8))
    return raw


@pytest.mark.parametrize("n", [0, 1, 3, 5, 9, 4099, 65536 + 13, (1 << 20) + 5])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("write_through", [False, True])
def test_fused_average_entry_point_vs_oracle(n, dtype, write_through):
    """dpwa_average -- the product kernel (device factor + lerp [+ the next snapshot]) over
    caller-owned buffers -- at ragged sizes: clock interpolation (interpolation.py:22-24) and
    the clock update of dpwa.py:150 against the oracle policy, the payload against the C oracle
    lerp, and the write-through copy equal to the averaged parameters."""
    rng = np.random.default_rng(1000 + n)
    p32 = rng.standard_normal(n).astype(np.float32)
    q32 = rng.standard_normal(n).astype(np.float32)
    my_clock, peer_clock = 3.0, 7.0
    f, new_clock = opolicy.factor_and_clock("clock", None, 0.0, my_clock, peer_clock, 1.0, 1.0)
    if dtype == "f32":
        exp = p32.copy()
        olerp.c_lerp_f32_(exp, q32, f)
        p, q = torch.from_numpy(p32).to(DEV), torch.from_numpy(q32).to(DEV)
    else:
        pu, qu = olerp.f32_to_bf16(p32), olerp.f32_to_bf16(q32)
        exp = pu.copy()
        olerp.c_lerp_bf16_(exp, qu, f)
        p, q = from_u16(pu), from_u16(qu)
    slot = average_slot(q, peer_clock, 1.0)
    snap = torch.full_like(p, float("nan")) if write_through else None
    clock = torch.tensor([my_clock, -1.0], dtype=torch.float64, device=DEV)
    coef = torch.zeros(32, dtype=torch.uint8, device=DEV)
    cfg = _lib.Interp(_lib.INTERP_CLOCK, 0, 0.0, 0.0)
    _lib.call("dpwa_average", _lib.F32 if dtype == "f32" else _lib.BF16, ptr(p), ptr(slot), n, ctypes.byref(cfg),
              ptr(clock), 1.0, ptr(coef), ptr(snap) if write_through else None, stream(), None, None)
    torch.cuda.synchronize()
    got = p.cpu().numpy() if dtype == "f32" else to_u16(p)
    assert olerp.bits_equal(got, exp)
    c = _lib.Coef.from_buffer_copy(coef.cpu().numpy().tobytes())
    assert c.status == 0 and c.factor == f
    assert clock[1].item() == new_clock      # dpwa.py:150
    if write_through and n:
        assert torch.equal(snap.view(torch.uint8), p.view(torch.uint8))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_average_zero_division_still_writes_the_snapshot(dtype):
    """Loss interpolation with loss + peer_loss == 0 raises ZeroDivisionError in the reference
    (interpolation.py:31-33): the parameters and clock stay, and a write-through snapshot
    still receives the (unchanged) parameters, ragged tail included."""
    n = 4099
    p = torch.randn(n, device=DEV).to(dtype)
    before = p.clone()
    slot = average_slot(torch.randn(n, device=DEV).to(dtype), 5.0, 0.0)
    snap = torch.zeros_like(p)
    clock = torch.tensor([2.0, -1.0], dtype=torch.float64, device=DEV)
    coef = torch.zeros(32, dtype=torch.uint8, device=DEV)
    cfg = _lib.Interp(_lib.INTERP_LOSS, 0, 0.0, 0.0)
    _lib.call("dpwa_average", _lib.F32 if dtype == torch.float32 else _lib.BF16, ptr(p), ptr(slot), n,
              ctypes.byref(cfg), ptr(clock), 0.0, ptr(coef), ptr(snap), stream(), None, None)
    torch.cuda.synchronize()
    assert _lib.Coef.from_buffer_copy(coef.cpu().numpy().tobytes()).status == _lib.STATUS_ZERO_DIVISION
    assert torch.equal(p, before) and torch.equal(snap, before)
    assert clock[1].item() == 2.0


@pytest.mark.parametrize("nr,nw", [(1, 1), (1, 2), (2, 1), (2, 2)])
def test_stream_mix_measurement_kernel(nr, nw):
    """dpwa_stream_mix (bench.py's roofline.mix_ceiling, not a product path): every 32-bit word of
    the destinations is the wrap-around sum of the sources' words, over an exact grid of 1-KiB
    spans whose last one is partial; bytes past nbytes are untouched; the first destination may be
    a source (in place, as the bench runs it)."""
    nbytes = 5 * 1024 + 48
    words = nbytes // 4
    src = [torch.randint(-2**31, 2**31 - 1, (words + 16,), dtype=torch.int32, device=DEV) for _ in range(nr)]
    dst = [torch.full((words + 16,), 7, dtype=torch.int32, device=DEV) for _ in range(nw)]
    dst[0] = src[-1] if nr == 2 else dst[0]          # in place when two sources
    want = src[0].cpu().numpy().astype(np.int64)[:words]
    if nr == 2:
        want = want + src[1].cpu().numpy().astype(np.int64)[:words]
    want = ((want + 2**31) % 2**32 - 2**31).astype(np.int32)
    tail = [d.cpu().numpy()[words:].copy() for d in dst]
    d_arr = (ctypes.c_void_p * 2)(*[d.data_ptr() for d in dst])
    s_arr = (ctypes.c_void_p * 2)(*[x.data_ptr() for x in src])
    _lib.call("dpwa_stream_mix", d_arr, nw, s_arr, nr, nbytes, stream(), None, None)
    torch.cuda.synchronize()
    for d, t in zip(dst, tail):
        got = d.cpu().numpy()
        assert np.array_equal(got[:words], want)
        assert np.array_equal(got[words:], t)
    with pytest.raises(_lib.DpwaError):
        _lib.call("dpwa_stream_mix", d_arr, nw, s_arr, nr, nbytes + 4, stream(), None, None)
