"""Multi-process gossip through the production DistGroup path on the GPU box: two ranks
share the one GPU, map each other's snapshot slots with hipIpcOpenMemHandle and pull them
on their side streams, lock-step, checked against the oracle simulation.  (RCCL refuses
two ranks on one device, so the barrier runs over gloo here; the data path -- IPC-mapped
slots, side-stream pulls, device factor, fused lerp -- is the production one.)"""
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import gossip as ogossip
from oracle import lerp as olerp
from tests import dist_worker

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,interp,fp,thr,pull", [(2, "clock", 1.0, 0.0, "copy"), (3, "loss", 0.7, 0.5, "copy"),
                                                       (2, "constant", 1.0, 0.0, "kernel:64"),
                                                       (3, "clock", 0.7, 0.0, "kernel"),
                                                       (2, "clock", 1.0, 0.0, "relay:8"),
                                                       (3, "loss", 0.7, 0.5, "relay"),
                                                       (4, "clock", 0.6, 0.0, "relay:16"),
                                                       (2, "clock", 1.0, 0.0, "relay-avg:8"),
                                                       (3, "loss", 0.7, 0.5, "relay-avg"),
                                                       (4, "clock", 0.6, 0.0, "relay-avg:16")])
def test_ipc_gossip_matches_oracle(tmp_path, world, interp, fp, thr, pull, n=100_003, dtype="f32"):
    T = 12
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "dist.yaml")
    dist_worker.write_cfg(cfg, names, fp, interp, thr)
    mp.spawn(dist_worker.gossip_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, "gloo", 0, pull, dtype),
             nprocs=world, join=True)
    init, deltas, send, wait = dist_worker.inputs(world, n, T, dtype=dtype)
    kw = dict(lerp=olerp.lerp_bf16, add=ogossip.add_bf16) if dtype == "bf16" else {}
    exp = ogossip.simulate(names, init, deltas, send, wait, interp, 0.5, thr, fp, [500 + r for r in range(world)],
                           **kw)
    for r in range(world):
        got = np.load(tmp_path / ("rank%d.npz" % r))
        want_peers = [p[0] if p else "" for p in (exp["picks"][t][r] for t in range(T))]
        assert list(got["peers"]) == want_peers, r
        assert np.array_equal(got["clocks"], exp["clocks"][:, r]), r
        assert olerp.bits_equal(got["params"], exp["params"][:, r]), r


@pytest.mark.parametrize("world,interp,fp,thr,pull", [(2, "clock", 1.0, 0.0, "copy"),
                                                       (3, "loss", 0.7, 0.5, "kernel:64"),
                                                       (3, "clock", 0.8, 0.0, "relay:8"),
                                                       (3, "clock", 0.8, 0.0, "relay-avg:8")])
def test_ipc_gossip_bf16_matches_oracle(tmp_path, world, interp, fp, thr, pull):
    """bf16 through every pull (BASELINE configs[3-4] dtype) with an odd element count: the
    payload (2n bytes) is not a multiple of the 16-byte vector, so the copy engine, the pull
    kernel and the relay's stripes all handle a ragged tail; bit-exact against the oracle's
    torch-eager bf16 lerp and bf16 training-step add."""
    test_ipc_gossip_matches_oracle(tmp_path, world, interp, fp, thr, pull, n=100_003, dtype="bf16")


@pytest.mark.parametrize("world,interp,fp,thr,pull,dtype", [(2, "clock", 1.0, 0.0, "copy", "f32"),
                                                             (3, "loss", 0.7, 0.5, "kernel:64", "bf16"),
                                                             (3, "clock", 0.7, 0.0, "relay:8", "f32"),
                                                             (3, "clock", 0.8, 0.0, "relay-avg:8", "bf16"),
                                                             (2, "constant", 1.0, 0.0, "relay-avg:8", "f32")])
def test_ipc_gossip_resident_matches_oracle(tmp_path, world, interp, fp, thr, pull, dtype, n=100_003):
    """Resident learners (parameters in their IPC-exported slots; the average reads the published
    slot and writes the other) in separate processes through every pull, the relay's fused
    out-of-place average included, f32 and bf16 with a ragged payload, rounds without a fetch
    relocating: parameters, clocks and peers bit-exact with oracle/gossip.py in the resident loop
    order (the step after update_wait)."""
    T = 10
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "res.yaml")
    dist_worker.write_cfg(cfg, names, fp, interp, thr)
    mp.spawn(dist_worker.gossip_worker,
             args=(world, free_port(), cfg, str(tmp_path), n, T, "gloo", 0, pull, dtype, False, True),
             nprocs=world, join=True)
    init, deltas, send, wait = dist_worker.inputs(world, n, T, dtype=dtype)
    kw = dict(lerp=olerp.lerp_bf16, add=ogossip.add_bf16) if dtype == "bf16" else {}
    exp = ogossip.simulate(names, init, deltas, send, wait, interp, 0.5, thr, fp, [500 + r for r in range(world)],
                           train_after_wait=True, **kw)
    for r in range(world):
        got = np.load(tmp_path / ("rank%d.npz" % r))
        want_peers = [p[0] if p else "" for p in (exp["picks"][t][r] for t in range(T))]
        assert list(got["peers"]) == want_peers, r
        assert np.array_equal(got["clocks"], exp["clocks"][:, r]), r
        assert olerp.bits_equal(got["params"], exp["params"][:, r]), r


@pytest.mark.parametrize("pull", ["copy", "relay:64", "relay-avg:64"])
def test_ipc_gossip_configs2_full_size(tmp_path, pull):
    """BASELINE configs[2] at its own size and interpolation through the multi-process path:
    100,000,000 fp32 per rank, clock interpolation, lock-step rounds over IPC-mapped slots
    (here two ranks share the one GPU); every round's parameters compared with the oracle by
    sha1 of the whole vector, clocks and peers exactly."""
    import hashlib
    world, n, T = 2, 100_000_000, 3
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "c2.yaml")
    dist_worker.write_cfg(cfg, names, 1.0, "clock", 0.0)
    mp.spawn(dist_worker.gossip_worker,
             args=(world, free_port(), cfg, str(tmp_path), n, T, "gloo", 0, pull, "f32", True), nprocs=world, join=True)
    init, deltas, send, wait = dist_worker.inputs(world, n, T)
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", 0.5, 0.0, 1.0, [500 + r for r in range(world)])
    for r in range(world):
        got = np.load(tmp_path / ("rank%d.npz" % r))
        assert list(got["peers"]) == [p[0] if p else "" for p in (exp["picks"][t][r] for t in range(T))], r
        assert np.array_equal(got["clocks"], exp["clocks"][:, r]), r
        want = [hashlib.sha1(exp["params"][t, r].tobytes()).hexdigest() for t in range(T)]
        assert list(got["params"]) == want, r


@pytest.mark.parametrize("n,interp,fp,thr,pull", [(1_000_000_000, "loss", 1.0, 0.5, "relay:128"),
                                                  (1_000_000_000, "loss", 1.0, 0.5, "relay-avg:128"),
                                                  (7_000_000_000, "constant", 0.7, 0.0, "copy"),
                                                  (7_000_000_000, "constant", 0.7, 0.0, "kernel:512")])
def test_ipc_gossip_configs3_4_full_size(tmp_path, n, interp, fp, thr, pull):
    """BASELINE configs[3] (1B bf16, loss interpolation, divergence_threshold 0.5 crossed by a
    decaying loss) and configs[4] (7B bf16, fetch_probability 0.7) at full size through the
    multi-process path: two ranks over IPC-mapped slots (byte offsets beyond 2^32), split and
    fused write-through rounds; sampled windows of every round's parameters (head, middle,
    ragged tail) bit-exact against the oracle replaying those windows, clocks and peers exact."""
    world, T = 2, 4
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "big.yaml")
    dist_worker.write_cfg(cfg, names, fp, interp, thr)
    mp.spawn(dist_worker.big_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, pull, "bf16"),
             nprocs=world, join=True)
    idx = np.concatenate([np.arange(b, e, dtype=np.int64) for b, e in dist_worker.synth_windows(n)])
    init = np.stack([olerp.f32_to_bf16(dist_worker.synth_f32(idx, g, -1)) for g in range(world)])
    deltas = np.stack([np.stack([olerp.f32_to_bf16(dist_worker.synth_f32(idx, g, r)) for g in range(world)])
                       for r in range(T)])
    send, wait = dist_worker.synth_losses(world, T)
    exp = ogossip.simulate(names, init, deltas, send, wait, interp, 0.5, thr, fp, [500 + r for r in range(world)],
                           lerp=olerp.lerp_bf16, add=ogossip.add_bf16)
    for r in range(world):
        got = np.load(tmp_path / ("rank%d.npz" % r))
        assert list(got["peers"]) == [p[0] if p else "" for p in (exp["picks"][t][r] for t in range(T))], r
        assert np.array_equal(got["clocks"], exp["clocks"][:, r]), r
        assert olerp.bits_equal(got["params"], exp["params"][:, r]), r


@pytest.mark.parametrize("pull", ["relay:8", "relay-avg:8", "kernel"])
def test_ipc_gossip_six_ranks(tmp_path, monkeypatch, pull):
    """Six ranks (the relay's stripes over more than four peers).  Six processes on one card
    oversubscribe its hardware queues with the default 4 per process, so the children get 2."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    test_ipc_gossip_matches_oracle(tmp_path, 6, "clock", 0.8, 0.0, pull, n=65_537)


@pytest.mark.parametrize("pull", ["relay:2", "relay-avg:2"])
def test_relay_tiny_payload(tmp_path, pull):
    """5 parameters over 4 ranks: one stripe holding all 20 bytes, three empty ones (the fused
    form reads one 16-B item and a one-element ragged tail from that stripe)."""
    test_ipc_gossip_matches_oracle(tmp_path, 4, "constant", 1.0, 0.0, pull, n=5)


@pytest.mark.parametrize("pull", ["copy", "relay:8", "relay-avg:8"])
def test_ipc_gossip_with_injected_faults(tmp_path, pull):
    """Remote peers marked slow (timeouts), down (refused) or dead (removed) steer the
    native scheduler exactly as the reference's TxThread: checked against the oracle fed
    the same outcomes (conn.py:246-313)."""
    world, n, T = 3, 50_001, 10
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "faults.yaml")
    dist_worker.write_cfg(cfg, names, 1.0, "clock", 0.0)
    mp.spawn(dist_worker.fault_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, pull), nprocs=world,
             join=True)
    init, deltas, send, wait = dist_worker.inputs(world, n, T)
    from oracle.policy import OracleLearner
    learners = [OracleLearner(names[g], [x for x in names if x != names[g]], 1.0, "clock", None, 0.0, 500 + g)
                for g in range(world)]
    params = init.copy()
    faults = [{} for _ in range(world)]
    for r in range(T):
        states, snaps = [], []
        for g in range(world):
            for peer, f in dist_worker.FAULTS.get(g, {}).get(r, {}).items():
                if f is None:
                    faults[g].pop(peer, None)
                else:
                    faults[g][peer] = f
            states.append(learners[g].update_send(send[r][g]))
            snaps.append(params[g].copy())
        for g in range(world):
            params[g] = np.add(params[g], deltas[r, g], dtype=np.float32)
        for g in range(world):
            fl = faults[g]
            conn_fn = lambda p, fl=fl: {"down": "refused", "dead": "error"}.get(fl.get(p), "ok")
            req_fn = lambda p, fl=fl: ({"slow": ("timeout", None, None), "dead": ("error", None, None),
                                        "down": ("error", None, None)}.get(fl.get(p)) or
                                       ("payload", states[names.index(p)], snaps[names.index(p)]))
            st, pl, att = learners[g].fetch(conn_fn, req_fn) if learners[g].fetching else (None, None, [])
            averaged, f = learners[g].update_wait(wait[r][g], st, pl is not None)
            if averaged:
                params[g] = olerp.lerp_f32(params[g], pl, f)
            got = np.load(tmp_path / ("rank%d.npz" % g))
            want_peer = att[-1]["peer"] if pl is not None else ""
            assert got["peers"][r] == want_peer, (g, r)
            assert got["clocks"][r] == learners[g].clock, (g, r)
            assert olerp.bits_equal(got["params"][r], params[g]), (g, r)
            want_scores = [-1 if s is None else s for s in learners[g].scores([x for x in names if x != names[g]])]
            assert list(got["scores"][r]) == want_scores, (g, r)


@pytest.mark.parametrize("world,interp,fp,thr,pull", [(2, "clock", 1.0, 0.0, "copy"), (3, "loss", 0.7, 0.5, "kernel:64"),
                                                       (3, "clock", 0.8, 0.0, "relay:8"),
                                                       (3, "clock", 0.8, 0.0, "relay-avg:8")])
def test_ipc_gossip_vmm_shared_slots(tmp_path, monkeypatch, world, interp, fp, thr, pull):
    """DPWA_VMM=1: the snapshot slots (and relay buffers) are hipMemCreate chunks shared as fds
    over a Unix socket -- the form every allocation of 1.5 GiB and more takes, since
    hipIpcOpenMemHandle does not return above ~2 GiB -- at a small size, against the oracle."""
    monkeypatch.setenv("DPWA_VMM", "1")
    test_ipc_gossip_matches_oracle(tmp_path, world, interp, fp, thr, pull, n=100_003)
