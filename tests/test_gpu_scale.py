"""bf16 end-to-end parity and BASELINE-size gossip rounds (configs 3-5: 100M fp32,
1B bf16, 7B bf16) on one GPU, through the drop-in API.

At full size the check is size-independent: with constant interpolation 0.5 and two
learners that average each other's snapshots of the same round, the two results must be
bit-identical (a*q + b*p == a*p + b*q when a == b), they must equal torch-eager
`f*t + (1-f)*p` on sampled windows, and an f = 0 round must leave the parameters
untouched (identity)."""
import numpy as np
import pytest
import torch

from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter
from dpwa_amd.group import LocalGroup
from oracle import gossip as ogossip
from oracle import lerp as olerp
from tests.test_gpu_gossip import Net, write_cfg

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def test_bf16_adapter_gossip_matches_oracle(tmp_path):
    rng = np.random.default_rng(21)
    G, T = 4, 10
    shapes = [(33, 17), (17,), (1000,), (3, 5, 7)]
    n = sum(int(np.prod(s)) for s in shapes)
    names = ["b%d" % g for g in range(G)]
    init32 = rng.standard_normal((G, n)).astype(np.float32)
    init = olerp.f32_to_bf16(init32).reshape(G, n)
    send = [[float(2 - 0.1 * r + 0.01 * g) for g in range(G)] for r in range(T)]
    wait = [[float(2 - 0.1 * r - 0.01 * g) for g in range(G)] for r in range(T)]
    seeds = [60 + g for g in range(G)]
    deltas = np.zeros((T, G, n), np.uint16)            # bf16 bits: averaging only
    exp = ogossip.simulate(names, init, deltas, send, wait, "loss", None, 0.0, 0.9, seeds, lerp=olerp.lerp_bf16)
    cfg = tmp_path / "bf16.yaml"
    write_cfg(cfg, names, 0.9, "loss", 0.0, None)
    group = LocalGroup()
    nets, adapters = [], []
    for g in range(G):
        net = Net(shapes, dtype=torch.bfloat16).to(DEV)
        flat = torch.from_numpy(init[g].view(np.int16)).view(torch.bfloat16)
        off = 0
        with torch.no_grad():
            for _, p in net.named_parameters():
                k = p.numel()
                p.copy_(flat[off:off + k].view(p.shape))
                off += k
        nets.append(net)
        adapters.append(DpwaPyTorchAdapter(net, names[g], str(cfg), seed=seeds[g], group=group))
    for r in range(T):
        for g in range(G):
            adapters[g].update_send(send[r][g])
        for g in range(G):
            adapters[g].update_wait(wait[r][g])
    for g in range(G):
        got = torch.cat([p.detach().reshape(-1) for _, p in nets[g].named_parameters()])
        got = got.view(torch.int16).cpu().numpy().view(np.uint16)
        assert olerp.bits_equal(got, exp["params"][-1, g]), g
        assert adapters[g].connection.clock == exp["clocks"][-1, g]


@pytest.mark.parametrize("n,dtype", [(100_000_000, torch.float32), (1_000_000_000, torch.bfloat16),
                                     (7_000_000_000, torch.bfloat16)])
def test_full_size_gossip_round(tmp_path, n, dtype):
    cfg = tmp_path / "big.yaml"
    write_cfg(cfg, ["A", "B"], 1.0, "constant", 0.0, 0.5)
    group = LocalGroup()
    g = torch.Generator(device=DEV).manual_seed(n % 1000)
    flats = []
    for _ in range(2):
        t = torch.empty(n, dtype=dtype, device=DEV)
        chunk = 1 << 28
        for s in range(0, n, chunk):                        # fp32 randn in chunks, then cast
            e = min(n, s + chunk)
            t[s:e] = torch.randn(e - s, device=DEV, generator=g).to(dtype)
        flats.append(t)
    win = [slice(0, 1 << 20), slice(n // 2, n // 2 + 4099), slice(n - (1 << 20) - 3, n)]
    before = [[f[w].clone() for w in win] for f in flats]
    conns = [DpwaConnection(nm, str(cfg), seed=1 + i, group=group) for i, nm in enumerate(["A", "B"])]
    for c, f in zip(conns, flats):
        c.update_send(f, 1.0)
    for c, f in zip(conns, flats):
        payload, _ = c.update_wait_average(f, 1.0)
        assert payload is not None
    torch.cuda.synchronize()
    iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
    assert torch.equal(flats[0].view(iv), flats[1].view(iv))          # symmetric at f = 0.5
    for k, w in enumerate(win):
        p, q = before[0][k], before[1][k]
        want = 0.5 * q + (1 - 0.5) * p                                    # torch eager, same device
        assert torch.equal(flats[0][w].view(iv), want.view(iv))
    for c in conns:
        assert c.clock == 1.0
        c.close()
    del flats, before
    torch.cuda.empty_cache()
