"""BASELINE.json's configs, each at its own size and with its own settings, on one GPU through
the drop-in API, checked against the oracle (oracle/ is pinned to the reference's fixtures).

* configs[0]: four CIFAR ResNet-18 learners (62 tensors, 11,173,962 parameters) training on
  synthetic batches (SGD lr 0.01, momentum 0.9, wd 5e-4, batch 8: prepare.py:31, main.py:
  122-158) with constant 0.5 interpolation, fetch_probability 1 and divergence_threshold 0.5
  (dpwa.yaml.t:6-19).  Every averaging is checked against oracle.lerp of the learner's own
  parameters just before update_wait and the peer's published snapshot, with the peer, factor
  and clock from oracle.policy.
* configs[1]: exactly 11,173,962 fp32 per learner through DpwaPyTorchAdapter, compared with
  the C oracle over the whole vector, at factors 0.5 and 1/3.
* configs[2-4] at full size (100M fp32 clock interpolation; 1B bf16 loss interpolation with
  divergence_threshold 0.5 and a decaying loss that crosses it; 7B bf16 fetch_probability 0.7
  with flow control): peers, clocks and factors every round against oracle.policy, and the
  averaged values on sampled windows against the oracle lerp (fp32: bit-exact; bf16: the
  torch-eager two-rounding form, bit-exact)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter
from dpwa_amd.group import LocalGroup
from oracle import lerp as olerp
from oracle.policy import OracleLearner
from tests.test_gpu_gossip import write_cfg

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
RESNET18_NUMEL = 11_173_962


def resnet18():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
    from resnet18_gossip import resnet18 as make
    return make()


def oracle_round(L, send, wait, names):
    """One lock-step round of the oracle learners: returns per learner (peer index or None,
    factor)."""
    states = [L[g].update_send(send[g]) for g in range(len(L))]
    out = []
    for g in range(len(L)):
        if not L[g].fetching:
            L[g].update_wait(wait[g], None, False)
            out.append((None, 0.0))
            continue
        st, payload, att = L[g].fetch(lambda p: "ok", lambda p: ("payload", states[names.index(p)], b"x"))
        _, factor = L[g].update_wait(wait[g], st, payload is not None)
        out.append((names.index(att[-1]["peer"]), factor))
    return out


def test_configs0_resnet18_four_learners_training(tmp_path):
    G, T = 4, 6
    names = ["w%d" % (g + 1) for g in range(G)]
    cfg = tmp_path / "c0.yaml"
    write_cfg(cfg, names, 1, "constant", 0.5, 0.5)
    torch.manual_seed(0)
    nets = [resnet18().to(DEV) for _ in range(G)]
    assert sum(p.numel() for p in nets[0].parameters()) == RESNET18_NUMEL
    assert len(list(nets[0].parameters())) == 62
    opts = [torch.optim.SGD(n.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4) for n in nets]
    group = LocalGroup()
    adapters = [DpwaPyTorchAdapter(nets[g], names[g], str(cfg), seed=100 + g, group=group) for g in range(G)]
    L = [OracleLearner(names[g], [x for x in names if x != names[g]], 1, "constant", 0.5, 0.5, 100 + g)
         for g in range(G)]
    gen = torch.Generator(device=DEV).manual_seed(5)
    send = [2.3] * G
    for r in range(T):
        for g in range(G):
            adapters[g].update_send(send[g])
        snaps = [a.flat.buffer.cpu().numpy() for a in adapters]         # what each learner published
        wait = []
        for g in range(G):                                               # main.py:134-139
            x = torch.randn(8, 3, 32, 32, device=DEV, generator=gen)
            y = torch.randint(0, 10, (8,), device=DEV, generator=gen)
            opts[g].zero_grad(set_to_none=True)
            loss = F.cross_entropy(nets[g](x), y)
            loss.backward()
            opts[g].step()
            wait.append(loss.item() * (0.1 if r >= 3 else 1.0))         # from round 3 below the threshold
        before = [a.flat.buffer.cpu().numpy() for a in adapters]
        for g in range(G):
            adapters[g].update_wait(wait[g])
        exp = oracle_round(L, send, wait, names)
        for g in range(G):
            q, factor = exp[g]
            got = adapters[g].flat.buffer.cpu().numpy()
            assert adapters[g].connection.last_fetch_peer == names[q], (r, g)
            assert olerp.bits_equal(got, olerp.lerp_f32(before[g], snaps[q], factor)), (r, g)
            assert adapters[g].connection.clock == L[g].clock, (r, g)
        send = wait
    for a in adapters:
        a.connection.close()


def test_configs1_resnet_size_adapter_round_matches_c_oracle(tmp_path):
    for value in (0.5, 1.0 / 3.0):
        cfg = tmp_path / "c1.yaml"
        write_cfg(cfg, ["A", "B"], 1, "constant", 0.0, value)
        group = LocalGroup()

        class Flat(torch.nn.Module):
            def __init__(self, seed):
                super().__init__()
                g = torch.Generator(device=DEV).manual_seed(seed)
                self.w = torch.nn.Parameter(torch.randn(RESNET18_NUMEL, device=DEV, generator=g))

        nets = [Flat(0).to(DEV), Flat(1).to(DEV)]
        adapters = [DpwaPyTorchAdapter(nets[i], nm, str(cfg), seed=i, group=group) for i, nm in enumerate("AB")]
        assert adapters[0].flat.numel == RESNET18_NUMEL + (-RESNET18_NUMEL % 64)
        want = [n.w.detach().cpu().numpy().copy() for n in nets]
        for r in range(3):
            for a in adapters:
                a.update_send(1.0)
            snaps = [w.copy() for w in want]
            for i, a in enumerate(adapters):
                a.update_wait(1.0)
                olerp.c_lerp_f32_(want[i], snaps[1 - i], value)
            for i in range(2):
                assert olerp.bits_equal(nets[i].w.detach().cpu().numpy(), want[i]), (value, r, i)
        for a in adapters:
            a.connection.close()
        del nets, adapters
        torch.cuda.empty_cache()


def _fill(n, dtype, seed):
    t = torch.empty(n, dtype=dtype, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(seed)
    chunk = 1 << 28
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        t[s:e] = torch.randn(e - s, device=DEV, generator=g).to(dtype)
    return t


def _bits(t):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    return t.cpu().numpy()


@pytest.mark.parametrize("cfgname,n,dtype,G,interp,fp,thr,T", [
    ("configs[2]", 100_000_000, torch.float32, 3, "clock", 1, 0.0, 6),
    ("configs[3]", 1_000_000_000, torch.bfloat16, 2, "loss", 1, 0.5, 8),
    ("configs[4]", 7_000_000_000, torch.bfloat16, 3, "constant", 0.7, 0.0, 5),
])
def test_full_size_configs_with_their_settings(tmp_path, cfgname, n, dtype, G, interp, fp, thr, T):
    names = ["w%d" % (g + 1) for g in range(G)]
    cfg = tmp_path / "big.yaml"
    write_cfg(cfg, names, fp, interp, thr, 0.5)
    group = LocalGroup()
    flats = [_fill(n, dtype, 10 + g) for g in range(G)]
    conns = [DpwaConnection(names[g], str(cfg), seed=300 + g, group=group) for g in range(G)]
    L = [OracleLearner(names[g], [x for x in names if x != names[g]], fp, interp, 0.5, thr, 300 + g)
         for g in range(G)]
    win = [slice(0, 1 << 16), slice(n // 2 - 7, n // 2 + 4099), slice(n - (1 << 16) - 3, n)]
    lerp = olerp.lerp_bf16 if dtype == torch.bfloat16 else olerp.lerp_f32
    rng = np.random.default_rng(8)
    crossed = False
    for r in range(T):
        # SURVEY §8d C4's loss 2 exp(-t/200) + 0.05 U(0,1), time-compressed (t/3) so that it
        # crosses the 0.5 divergence threshold within the run
        send = [2.0 * float(np.exp(-r / 3.0)) + 0.05 * float(rng.random()) for _ in range(G)]
        wait = [2.0 * float(np.exp(-(r + 0.5) / 3.0)) + 0.05 * float(rng.random()) for _ in range(G)]
        crossed |= min(wait) < thr
        for g in range(G):
            conns[g].update_send(flats[g], send[g], reuse_snapshot=r % 2 == 1)
        snaps = [[_bits(f[w]) for w in win] for f in flats]
        exp = oracle_round(L, send, wait, names)
        for g in range(G):
            payload, _ = conns[g].update_wait_average(flats[g], wait[g], write_through=r % 2 == 0)
            q, factor = exp[g]
            assert (payload.peer if payload is not None else None) == (names[q] if q is not None else None), (r, g)
            if q is not None:
                for k, w in enumerate(win):
                    got = _bits(flats[g][w])
                    assert olerp.bits_equal(got, lerp(snaps[g][k], snaps[q][k], factor)), (cfgname, r, g, k)
            else:
                for k, w in enumerate(win):
                    assert olerp.bits_equal(_bits(flats[g][w]), snaps[g][k]), (cfgname, r, g, k)
            assert conns[g].clock == L[g].clock, (cfgname, r, g)
        assert [conns[g].flow_control_scores() for g in range(G)] == \
               [dict(zip([x for x in names if x != names[g]], L[g].scores([x for x in names if x != names[g]])))
                for g in range(G)]
    if thr > 0:
        assert crossed
    for c in conns:
        c.close()
    del flats
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfgname,n,dtype,G,interp,fp,thr,T", [
    ("configs[2]", 100_000_000, torch.float32, 3, "clock", 1, 0.0, 5),
    ("configs[3]", 1_000_000_000, torch.bfloat16, 2, "loss", 1, 0.5, 8),
    ("configs[4]", 7_000_000_000, torch.bfloat16, 3, "constant", 0.7, 0.0, 6),
])
def test_full_size_configs_resident(tmp_path, cfgname, n, dtype, G, interp, fp, thr, T):
    """The same configs at full size with resident learners (the bench's form), their averages
    batched: sampled windows of every learner's parameters after every round against the oracle
    lerp of the published windows (a learner without a fetch keeps its parameters: relocated);
    peers, clocks and flow-control scores against the oracle policy; the served snapshot untouched
    by the round's averages."""
    names = ["w%d" % (g + 1) for g in range(G)]
    cfg = tmp_path / "bigres.yaml"
    write_cfg(cfg, names, fp, interp, thr, 0.5)
    group = LocalGroup()
    conns = [DpwaConnection(names[g], str(cfg), seed=300 + g, group=group) for g in range(G)]
    for g in range(G):
        conns[g].make_resident(_fill(n, dtype, 10 + g))
    torch.cuda.empty_cache()
    L = [OracleLearner(names[g], [x for x in names if x != names[g]], fp, interp, 0.5, thr, 300 + g)
         for g in range(G)]
    win = [slice(0, 1 << 16), slice(n // 2 - 7, n // 2 + 4099), slice(n - (1 << 16) - 3, n)]
    lerp = olerp.lerp_bf16 if dtype == torch.bfloat16 else olerp.lerp_f32
    rng = np.random.default_rng(9)
    crossed, relocated = False, 0
    for r in range(T):
        send = [2.0 * float(np.exp(-r / 3.0)) + 0.05 * float(rng.random()) for _ in range(G)]
        wait = [2.0 * float(np.exp(-(r + 0.5) / 3.0)) + 0.05 * float(rng.random()) for _ in range(G)]
        crossed |= min(wait) < thr
        for g in range(G):
            conns[g].update_send(conns[g].parameters, send[g])
        published = [c.parameters for c in conns]
        snaps = [[_bits(f[w]) for w in win] for f in published]
        exp = oracle_round(L, send, wait, names)
        res = DpwaConnection.update_wait_average_many(conns, published, wait)
        for g in range(G):
            payload, _ = res[g]
            q, factor = exp[g]
            assert (payload.peer if payload is not None else None) == (names[q] if q is not None else None), (r, g)
            now = conns[g].parameters
            assert now.data_ptr() != published[g].data_ptr()
            relocated += q is None
            for k, w in enumerate(win):
                want = lerp(snaps[g][k], snaps[q][k], factor) if q is not None else snaps[g][k]
                assert olerp.bits_equal(_bits(now[w]), want), (cfgname, r, g, k)
                assert olerp.bits_equal(_bits(published[g][w]), snaps[g][k]), (cfgname, r, g, k)
            assert conns[g].clock == L[g].clock, (cfgname, r, g)
        assert [conns[g].flow_control_scores() for g in range(G)] == \
               [dict(zip([x for x in names if x != names[g]], L[g].scores([x for x in names if x != names[g]])))
                for g in range(G)]
    if thr > 0:
        assert crossed
    if fp < 1:
        assert relocated > 0
    for c in conns:
        c.close()
    del published
    torch.cuda.empty_cache()


def test_gpu_key_moves_the_model_onto_its_device(tmp_path):
    """f4: a node's gpu: key places its learner -- the adapter re-homes a model built on the
    CPU into a flat buffer on that GPU (before the optimizer exists, as main.py:109-116)."""
    from dpwa_amd.launch import write_config
    cfg = write_config(str(tmp_path / "gpu.yaml"), ["a", "b"], gpus=[0, 0])
    nets = [torch.nn.Linear(7, 3), torch.nn.Linear(7, 3)]
    group = LocalGroup()
    adapters = [DpwaPyTorchAdapter(n, nm, cfg, seed=i, group=group) for i, (n, nm) in enumerate(zip(nets, "ab"))]
    for n in nets:
        assert all(p.device == DEV for p in n.parameters())
    want = [torch.cat([p.detach().reshape(-1) for p in n.parameters()]).cpu().numpy() for n in nets]
    for a in adapters:
        a.update_send(1.0)
    for a in adapters:
        a.update_wait(1.0)
    got = [torch.cat([p.detach().reshape(-1) for p in n.parameters()]).cpu().numpy() for n in nets]
    assert olerp.bits_equal(got[0], olerp.lerp_f32(want[0], want[1], 0.5))
    for a in adapters:
        a.connection.close()


def test_configs0_resnet18_resident_training(tmp_path):
    """configs[0]'s four ResNet-18 learners with resident parameters (the adapter's resident=True,
    62 parameters re-pointed into the slots every round), the resident loop order: update_send,
    update_wait, then the training step (SGD with momentum and weight decay).  Every average is the
    oracle lerp of the learner's published parameters with its peer's (constant 0.5, divergence
    threshold 0.5 crossed from round 3), the peers and clocks are the oracle's, and the optimizer
    keeps training the re-pointed parameters."""
    G, T = 4, 6
    names = ["w%d" % (g + 1) for g in range(G)]
    cfg = tmp_path / "c0r.yaml"
    write_cfg(cfg, names, 1, "constant", 0.5, 0.5)
    torch.manual_seed(0)
    nets = [resnet18().to(DEV) for _ in range(G)]
    opts = [torch.optim.SGD(n.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4) for n in nets]
    group = LocalGroup()
    adapters = [DpwaPyTorchAdapter(nets[g], names[g], str(cfg), seed=100 + g, group=group, resident=True)
                for g in range(G)]
    L = [OracleLearner(names[g], [x for x in names if x != names[g]], 1, "constant", 0.5, 0.5, 100 + g)
         for g in range(G)]
    gen = torch.Generator(device=DEV).manual_seed(5)
    send = [2.3] * G
    homes = [set() for _ in range(G)]
    for r in range(T):
        for g in range(G):
            adapters[g].update_send(send[g])
        snaps = [a.flat.buffer.cpu().numpy() for a in adapters]         # what each learner published
        wait = [s * (0.1 if r >= 3 else 1.0) for s in send]
        DpwaPyTorchAdapter.update_wait_many(adapters, wait)
        exp = oracle_round(L, send, wait, names)
        for g in range(G):
            q, factor = exp[g]
            got = torch.cat([p.detach().reshape(-1) for p in nets[g].parameters()]).cpu().numpy()
            want = olerp.lerp_f32(snaps[g], snaps[q], factor)
            flat = adapters[g].flat
            want = np.concatenate([want[o:o + p.numel()] for p, o in zip(flat.params, flat.offsets)])
            assert adapters[g].connection.last_fetch_peer == names[q], (r, g)
            assert olerp.bits_equal(got, want), (r, g)
            assert adapters[g].connection.clock == L[g].clock, (r, g)
            homes[g].add(adapters[g].flat.buffer.data_ptr())
        send = []
        for g in range(G):                                               # the step, after update_wait
            x = torch.randn(8, 3, 32, 32, device=DEV, generator=gen)
            y = torch.randint(0, 10, (8,), device=DEV, generator=gen)
            opts[g].zero_grad(set_to_none=True)
            loss = F.cross_entropy(nets[g](x), y)
            loss.backward()
            opts[g].step()
            send.append(loss.item())
    assert all(len(h) == 2 for h in homes)
    for a in adapters:
        a.connection.close()


def test_resnet18_example_runs(capsys):
    """f1: examples/resnet18_gossip.py (the reference trainer's loop, main.py:122-158) runs end
    to end with gossip every step; the clock advanced every round (fetch_probability 1)."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
    import resnet18_gossip
    for extra in ([], ["--resident"]):
        resnet18_gossip.main(["--learners", "2", "--steps", "4", "--warmup", "2", "--batch-size", "8"] + extra)
        out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
        assert out["learners"] == 2 and out["final_clock"] == 2 + 3 * 4   # warmup + three gossip phases
        assert out["train_steps_per_s_per_learner_gossip"] > 0 and out["resident"] == bool(extra)


@pytest.mark.parametrize("group", ["lockstep", "async"])
def test_configs0_resnet18_training_across_processes(tmp_path, group):
    """configs[0]'s trainer (ResNet-18, constant 0.5, threshold 0.5) with one learner per
    process through the multi-process groups (IPC-mapped slots; two ranks share the one GPU):
    every fetched snapshot is byte-identical to what its peer published that round, every
    average is oracle.lerp(before, fetched, factor), and -- lock-step -- peers and clocks
    follow the oracle replay of the recorded losses."""
    import torch.multiprocessing as mp

    from tests import dist_worker
    from tests.test_gpu_ipc import free_port
    G, T = 2, 5
    names = ["w%d" % (g + 1) for g in range(G)]
    cfg = tmp_path / "c0mp.yaml"
    write_cfg(cfg, names, 1, "constant", 0.5, 0.5)
    mp.spawn(dist_worker.resnet_worker, args=(G, free_port(), str(cfg), str(tmp_path), T, group), nprocs=G,
             join=True)
    runs = [np.load(tmp_path / ("rank%d.npz" % g)) for g in range(G)]
    for g in range(G):
        assert all(runs[g]["ok"]), (g, list(runs[g]["ok"]))
        for r in range(T):
            peer = str(runs[g]["peers"][r])
            if peer:
                q = names.index(peer)
                # free-running: whichever of the peer's publishes the board handed out
                allowed = {str(runs[q]["published"][r])} if group == "lockstep" else \
                    {str(h) for h in runs[q]["published"]}
                assert str(runs[g]["fetched"][r]) in allowed, (g, r)
    if group == "lockstep":
        L = [OracleLearner(names[g], [x for x in names if x != names[g]], 1, "constant", 0.5, 0.5, 100 + g)
             for g in range(G)]
        for r in range(T):
            exp = oracle_round(L, [runs[g]["send"][r] for g in range(G)], [runs[g]["wait"][r] for g in range(G)],
                               names)
            for g in range(G):
                q, _ = exp[g]
                assert str(runs[g]["peers"][r]) == (names[q] if q is not None else ""), (r, g)
                assert runs[g]["clocks"][r] == L[g].clock, (r, g)
