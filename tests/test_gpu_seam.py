"""The DpwaConnection seam used the reference's way (dpwa.py:125-156 returns (payload, factor);
pytorch.py:64-68 then evaluates ``factor * t + (1 - factor) * param`` itself): the device
factor takes part in torch arithmetic and gives the same bits as the fused kernel and as the
reference adapter's lerp (fixture)."""
import numpy as np
import pytest
import torch

from dpwa_amd import DpwaConnection
from dpwa_amd.group import LocalGroup
from oracle import lerp as olerp
from tests.test_gpu_gossip import write_cfg

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("interp,value", [("constant", 1.0 / 3.0), ("clock", None), ("loss", None)])
def test_reference_style_arithmetic_matches_fused_average(tmp_path, interp, value):
    rng = np.random.default_rng(17)
    n = 300_007
    cfg = tmp_path / "seam.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, interp, 0.0, value)
    init = rng.standard_normal((2, n)).astype(np.float32)
    ref_flats, fused_flats = [], []
    for flats, seed0 in ((ref_flats, 1), (fused_flats, 1)):
        group = LocalGroup()
        conns = [DpwaConnection(nm, str(cfg), seed=seed0 + i, group=group) for i, nm in enumerate(["a", "b"])]
        fl = [torch.from_numpy(init[g]).to(DEV) for g in range(2)]
        for r in range(3):
            for g, c in enumerate(conns):
                c.update_send(fl[g], 1.0 + 0.25 * g + r)
            for g, c in enumerate(conns):
                if flats is ref_flats:
                    payload, factor = c.update_wait(0.5 + 0.1 * g + r)
                    if payload is not None:
                        t = payload.tensor()
                        fl[g] = factor * t + (1 - factor) * fl[g]      # pytorch.py:68, verbatim (rebinds)
                else:
                    c.update_wait_average(fl[g], 0.5 + 0.1 * g + r)
        torch.cuda.synchronize()
        flats.extend(f.cpu().numpy() for f in fl)
        for c in conns:
            c.close()
    for g in range(2):
        assert olerp.bits_equal(ref_flats[g], fused_flats[g]), g


def test_device_factor_behaves_like_the_float():
    from dpwa_amd.dpwa import DeviceFactor

    class FakeLearner:
        version = 3
        device = DEV
        _h = object()

        def __init__(self, f):
            self.f = f
            import ctypes
            self.handle = ctypes.c_void_p(1)

        def read_coef(self):
            class C:
                factor = self.f
            return C()

    f = 2.0 / 7.0
    d = DeviceFactor(FakeLearner(f))
    d._t = torch.tensor(f, dtype=torch.float64, device=DEV)        # what copy_factor would enqueue
    t = torch.randn(1000, device=DEV)
    p = torch.randn(1000, device=DEV)
    assert torch.equal(d * t + (1 - d) * p, f * t + (1 - f) * p)
    assert float(d) == f
    assert float(1 - d) == 1 - f and float(d / 2) == f / 2 and float(-d) == -f


def test_loss_given_as_float32_float64_tensor_or_number(tmp_path):
    """update_send/update_wait accept the loss as a Python number, a float64 or a float32
    device tensor (read in place by the kernels, widened exactly as float() does): the
    factors and clocks of a loss-interpolated run match the oracle whatever the mix."""
    from oracle.policy import factor_and_clock
    cfg = tmp_path / "loss.yaml"
    write_cfg(cfg, ["a", "b"], 1.0, "loss", 0.5, None)
    group = LocalGroup()
    conns = [DpwaConnection(nm, str(cfg), seed=i, group=group) for i, nm in enumerate("ab")]
    flats = [torch.zeros(1024, device=DEV), torch.ones(1024, device=DEV)]
    kinds = [lambda x: x, lambda x: torch.tensor(x, dtype=torch.float64, device=DEV),
             lambda x: torch.tensor(x, dtype=torch.float32, device=DEV)]
    clocks = [0.0, 0.0]
    for r in range(9):
        send = [float(np.float32(0.9 ** r + 0.1 * g)) for g in range(2)]
        wait = [float(np.float32(0.8 ** r + 0.05 * g)) for g in range(2)]
        for g, c in enumerate(conns):
            c.update_send(flats[g], kinds[(r + g) % 3](send[g]))
        pub = [clocks[g] + 1.0 for g in range(2)]
        for g, c in enumerate(conns):
            payload, factor = c.update_wait(kinds[(r + 2 * g + 1) % 3](wait[g]))
            c.average(flats[g])
            f, clocks[g] = factor_and_clock("loss", None, 0.5, pub[g], pub[1 - g], wait[g], send[1 - g])
            assert float(factor) == f, (r, g)
            assert c.clock == clocks[g], (r, g)
    for c in conns:
        c.close()
