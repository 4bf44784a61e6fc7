"""Host-side pieces of resident parameters that need no GPU: the DLPack view over memory the
library owns (dpwa_amd/devview.py, exercised here on host memory with DLPack's CPU device
type), FlatParameters.rehome (the adapter re-points every parameter into the slot they are in
after each update_wait), and the oracle's resident loop order (oracle/gossip.py
train_after_wait)."""
import gc

import numpy as np
import torch

from dpwa_amd import devview
from dpwa_amd.flat import FlatParameters
from oracle import gossip as ogossip


def test_device_tensor_shares_memory_and_calls_nothing_when_freed():
    a = np.arange(1000, dtype=np.float32)
    t = devview.device_tensor(a.ctypes.data, 1000, torch.float32, 0, device_type=devview.KDL_CPU)
    assert t.dtype == torch.float32 and t.shape == (1000,) and t.data_ptr() == a.ctypes.data
    t[7] = -3.0
    assert a[7] == -3.0
    b = np.zeros(64, dtype=np.uint16)
    tb = devview.device_tensor(b.ctypes.data, 64, torch.bfloat16, 0, device_type=devview.KDL_CPU)
    tb.fill_(1.0)
    assert b[0] == 0x3F80                                # bf16 1.0
    made = devview.made[0]
    del t, tb
    gc.collect()                                        # no deleter: torch drops the views quietly
    assert devview.made[0] == made
    t2 = devview.device_tensor(a.ctypes.data, 1000, torch.float32, 0, device_type=devview.KDL_CPU)
    assert t2[7].item() == -3.0 and devview.made[0] == made + 1


def test_device_tensor_refuses_what_it_cannot_describe():
    import pytest
    with pytest.raises(KeyError):
        devview.device_tensor(1 << 20, 4, torch.float64, 0, device_type=devview.KDL_CPU)
    with pytest.raises(ValueError):
        devview.device_tensor(0, 4, torch.float32, 0, device_type=devview.KDL_CPU)


def test_rehome_repoints_every_parameter_and_keeps_training():
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 33), torch.nn.Tanh(), torch.nn.Linear(33, 5))
    flat = FlatParameters(net.named_parameters())
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9)
    slots = [torch.empty(flat.numel), torch.empty(flat.numel)]
    x = torch.randn(4, 7)
    ref = None
    for r in range(4):
        nxt = slots[r % 2]
        nxt.copy_(flat.buffer)                     # what the resident average leaves in the next slot
        flat.rehome(nxt)
        assert flat.buffer is nxt
        for p, o in zip(flat.params, flat.offsets):
            assert nxt.data_ptr() <= p.data_ptr() < nxt.data_ptr() + 4 * flat.numel
            assert torch.equal(p.detach().reshape(-1), nxt[o:o + p.numel()])
        opt.zero_grad()
        net(x).square().sum().backward()
        opt.step()                                 # the optimizer trains the re-pointed parameters
        assert not torch.equal(nxt, slots[(r + 1) % 2]) or r == 0
        ref = nxt
    assert flat.resync() == 0 and torch.equal(flat.buffer, ref)
    assert len(flat._homes) == 2                   # one view list per slot, built once


def test_oracle_train_after_wait_is_the_resident_order():
    """With no training deltas both orders are the same gossip; with deltas the resident order
    applies round r's step after its average (out_params then hold the averaged values)."""
    names = ["a", "b", "c"]
    rng = np.random.default_rng(3)
    init = rng.standard_normal((3, 257)).astype(np.float32)
    zero = np.zeros((5, 3, 257), np.float32)
    send = [[1.0 + g + r for g in range(3)] for r in range(5)]
    wait = [[0.5 + g + r for g in range(3)] for r in range(5)]
    seeds = [11, 12, 13]
    a = ogossip.simulate(names, init, zero, send, wait, "clock", None, 0.0, 0.7, seeds)
    b = ogossip.simulate(names, init, zero, send, wait, "clock", None, 0.0, 0.7, seeds, train_after_wait=True)
    assert np.array_equal(a["params"], b["params"]) and np.array_equal(a["clocks"], b["clocks"])
    deltas = (0.1 * rng.standard_normal((5, 3, 257))).astype(np.float32)
    c = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, 0.7, seeds, train_after_wait=True)
    assert np.array_equal(c["clocks"], a["clocks"])      # the policy does not see the parameters
    assert not np.array_equal(c["params"], a["params"])


def test_resident_adapter_update_wait_before_any_update_send_is_a_noop(tmp_path):
    """As in the reference (update_wait without a fetch returns (None, 0) and the adapter leaves
    the parameters alone), a resident adapter's update_wait before its first update_send does
    nothing -- no binding, no GPU call."""
    from dpwa_amd import DpwaPyTorchAdapter
    from dpwa_amd.launch import write_config
    from dpwa_amd.group import LocalGroup
    cfg = write_config(str(tmp_path / "r.yaml"), ["a", "b"], interpolation="constant")
    net = torch.nn.Linear(3, 2)
    before = [p.detach().clone() for p in net.parameters()]
    ad = DpwaPyTorchAdapter(net, "a", cfg, seed=1, group=LocalGroup(), resident=True)
    ad.update_wait(1.0)
    DpwaPyTorchAdapter.update_wait_many([ad], [1.0])
    assert ad.connection.parameters is None
    assert all(torch.equal(p.detach(), b) for p, b in zip(net.parameters(), before))
    ad.connection.close()
