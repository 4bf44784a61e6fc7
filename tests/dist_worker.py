"""Worker process for the multi-process gossip tests (spawned; one rank per process).

Each rank runs one DpwaConnection on its node under torch.distributed (world size == number
of nodes): the lock-step DistGroup for the trajectory tests, the free-running AsyncDistGroup
(the default) for the board tests.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def inputs(world, n, T, seed=0, dtype="f32"):
    """Initial parameters, per-round training deltas and losses; bf16 as raw bits (uint16)."""
    rng = np.random.default_rng(seed)
    init = rng.standard_normal((world, n), dtype=np.float32)
    deltas = rng.standard_normal((T, world, n), dtype=np.float32)
    deltas *= np.float32(0.01)
    send = [[float(2 * np.exp(-r / 4) + 0.05 * rng.random()) for _ in range(world)] for r in range(T)]
    wait = [[float(2 * np.exp(-(r + .5) / 4) + 0.05 * rng.random()) for _ in range(world)] for r in range(T)]
    if dtype == "bf16":
        from oracle.lerp import f32_to_bf16
        init, deltas = f32_to_bf16(init), f32_to_bf16(deltas)
    return init, deltas, send, wait


def to_device(a, dev):
    """An fp32 array, or raw bf16 bits (uint16), as a device tensor of that dtype."""
    import torch
    if a.dtype == np.uint16:
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).to(dev).view(torch.bfloat16)
    return torch.from_numpy(a).to(dev)


def to_host(t):
    """Inverse of to_device."""
    import torch
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    return t.cpu().numpy()


def write_cfg(path, names, fp, interp, thr):
    lines = ["- nodes:"] + ["  - {name: %s, host: 127.0.0.1, port: %d}" % (nm, 45500 + i)
                            for i, nm in enumerate(names)]
    lines += ["- fetch_probability: %r" % fp, "- timeout_ms: 2500", "- interpolation: %s" % interp,
              "- divergence_threshold: %r" % thr, "- constant: { value: 0.5 }", "- clock: 0", "- loss: 0"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def gossip_worker(rank, world, port, cfg_path, out_dir, n, T, backend, device_of_rank, pull="copy", dtype="f32",
                  digest=False, resident=False):
    """Lock-step rounds through DistGroup; saves every round's parameters (or, with
    `digest`, their sha1 -- for full-size vectors), clock and peer.  `resident`: the parameters
    live in the learner's slots, every round averages fused and the training delta comes after
    update_wait (the saved parameters are those right after the average)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", device_of_rank(rank) if callable(device_of_rank) else device_of_rank)
    torch.cuda.set_device(dev)
    from dpwa_amd import DpwaConnection
    from dpwa_amd.group import DistGroup
    init, deltas, send, wait = inputs(world, n, T, dtype=dtype)
    names = ["r%d" % i for i in range(world)]
    conn = DpwaConnection(names[rank], cfg_path, seed=500 + rank, pull=pull, group="lockstep")
    assert type(conn._group) is DistGroup
    flat = to_device(init[rank], dev)
    params = [] if digest else np.zeros((T, n), init.dtype)
    clocks = np.zeros(T)
    peers = []
    if resident:
        conn.make_resident(flat)
        for r in range(T):
            conn.update_send(conn.parameters, send[r][rank])
            payload, _ = conn.update_wait_average(conn.parameters, wait[r][rank])
            peers.append(payload.peer if payload is not None else None)
            params[r] = to_host(conn.parameters)
            clocks[r] = conn.clock
            conn.parameters.add_(to_device(deltas[r, rank], dev))      # the step, after update_wait
    for r in range(0 if not resident else T, T):
        conn.update_send(flat, send[r][rank])
        flat.add_(to_device(deltas[r, rank], dev))
        if r % 2:
            payload, factor = conn.update_wait(wait[r][rank])      # split: factor kernel, then lerp
            if payload is not None:
                conn.average(flat)
        else:
            payload, factor = conn.update_wait_average(flat, wait[r][rank])   # fused (adapter path)
        if payload is not None:
            peers.append(payload.peer)
        else:
            peers.append(None)
        if digest:
            params.append(hashlib.sha1(to_host(flat).tobytes()).hexdigest())
        else:
            params[r] = to_host(flat)
        clocks[r] = conn.clock
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), params=params, clocks=clocks,
             peers=np.array([p or "" for p in peers]))
    torch.cuda.synchronize()
    dist.barrier()
    conn.close()
    dist.destroy_process_group()


FAULTS = {  # rank -> {round: {peer name: fault}}; applied before that round's update_send
    0: {2: {"r1": "slow"}, 5: {"r1": None}, 7: {"r2": "dead"}},
    1: {3: {"r0": "down"}, 6: {"r0": None}},
}


def fault_worker(rank, world, port, cfg_path, out_dir, n, T, pull="copy"):
    """Like gossip_worker, with scripted faults (FAULTS) injected into this rank's node."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dpwa_amd import DpwaConnection
    init, deltas, send, wait = inputs(world, n, T)
    names = ["r%d" % i for i in range(world)]
    conn = DpwaConnection(names[rank], cfg_path, seed=500 + rank, pull=pull, group="lockstep")
    flat = torch.from_numpy(init[rank]).to(dev)
    params, clocks, peers, scores = np.zeros((T, n), np.float32), np.zeros(T), [], []
    for r in range(T):
        for peer, f in FAULTS.get(rank, {}).get(r, {}).items():
            conn.inject_fault(peer, f)
        conn.update_send(flat, send[r][rank])
        flat.add_(torch.from_numpy(deltas[r, rank]).to(dev))
        payload, _ = conn.update_wait_average(flat, wait[r][rank])
        peers.append(payload.peer if payload is not None else "")
        params[r] = flat.cpu().numpy()
        clocks[r] = conn.clock
        scores.append([conn.flow_control_scores()[p] for p in names if p != names[rank]])
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), params=params, clocks=clocks, peers=np.array(peers),
             scores=np.array([[-1 if s is None else s for s in row] for row in scores]))
    torch.cuda.synchronize()
    dist.barrier()
    conn.close()
    dist.destroy_process_group()


from oracle.async_check import async_base, async_base_bf16, async_loss  # noqa: E402  (checker's published values)


def async_worker(rank, world, port, cfg_path, out_dir, n, T, pull="copy", die_rank=-1, die_round=-1):
    """Free-running gossip (AsyncDistGroup): every round sets the parameters to
    async_base(rank, r), publishes, sleeps a rank- and round-dependent time on the GPU and
    averages with whatever version of a peer the board hands out.  Records the peer, the
    version it read, the result and the clock; the test recomputes them from the bases."""
    import time
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dpwa_amd import DpwaConnection
    from dpwa_amd.group import AsyncDistGroup
    names = ["r%d" % i for i in range(world)]
    conn = DpwaConnection(names[rank], cfg_path, seed=700 + rank, group="async", pull=pull)
    assert isinstance(conn._group, AsyncDistGroup)
    rng = np.random.default_rng(rank)
    flat = torch.empty(n, device=dev, dtype=torch.float32)
    bases = [torch.from_numpy(async_base(rank, r, n)).to(dev) for r in range(T)]
    params, clocks, peers, versions, scores = np.zeros((T, n), np.float32), np.zeros(T), [], [], []
    for r in range(T):
        if rank == die_rank and r == die_round:
            torch.cuda.synchronize()
            conn._group.leave(conn)    # leaves mid-run (the board entry closes, its readers drain)
            os._exit(0)                # ... and dies: no close(), no barrier
        flat.copy_(bases[r])
        conn.update_send(flat, async_loss(rank, r))
        torch.cuda._sleep(int(rng.integers(0, 400_000)))     # uneven "training steps"
        payload, _ = conn.update_wait_average(flat, async_loss(rank, r, wait=True))
        peers.append(payload.peer if payload is not None else "")
        versions.append(conn._info()[2] if payload is not None else 0)
        params[r] = flat.cpu().numpy()
        clocks[r] = conn.clock
        scores.append([conn.flow_control_scores()[p] for p in names if p != names[rank]])
        if rank == 0 and r % 7 == 0:
            time.sleep(0.002)      # host-side jitter too
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), params=params, clocks=clocks, peers=np.array(peers),
             versions=np.array(versions, dtype=np.int64),
             scores=np.array([[-1 if s is None else s for s in row] for row in scores]))
    # no collective at the end either: a dead rank would never join it
    open(os.path.join(out_dir, "done%d" % rank), "w").close()
    while sum(os.path.exists(os.path.join(out_dir, "done%d" % q)) for q in range(world) if q != die_rank) < \
            world - (1 if die_rank >= 0 else 0):
        time.sleep(0.01)
    conn.close()
    os._exit(0)                    # skip the process-group teardown (the dead rank never joins it)


def async_wt_worker(rank, world, port, cfg_path, out_dir, n, T, pull="copy", dtype="f32"):
    """Free-running rounds with write-through snapshots: update_send publishes the parameters
    the last average left (the averaging kernel wrote that snapshot), the "training step" then
    sets the parameters to async_base(rank, r), and the average writes the next snapshot.
    Records what async_worker records; the test reconstructs every published snapshot from
    the publisher's own recorded results."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dpwa_amd import DpwaConnection
    names = ["r%d" % i for i in range(world)]
    conn = DpwaConnection(names[rank], cfg_path, seed=800 + rank, pull=pull)      # the default group
    rng = np.random.default_rng(rank + 10)
    base = async_base if dtype == "f32" else async_base_bf16
    flat = to_device(base(rank, -1, n), dev)
    bases = [to_device(base(rank, r, n), dev) for r in range(T)]
    params, clocks, peers, versions = np.zeros((T, n), base(rank, 0, 1).dtype), np.zeros(T), [], []
    for r in range(T):
        conn.update_send(flat, async_loss(rank, r), reuse_snapshot=True)
        flat.copy_(bases[r])
        torch.cuda._sleep(int(rng.integers(0, 400_000)))
        payload, _ = conn.update_wait_average(flat, async_loss(rank, r, wait=True), write_through=True)
        peers.append(payload.peer if payload is not None else "")
        versions.append(conn._info()[2] if payload is not None else 0)
        params[r] = to_host(flat)
        clocks[r] = conn.clock
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), params=params, clocks=clocks, peers=np.array(peers),
             versions=np.array(versions, dtype=np.int64))
    open(os.path.join(out_dir, "done%d" % rank), "w").close()
    import time
    while sum(os.path.exists(os.path.join(out_dir, "done%d" % q)) for q in range(world)) < world:
        time.sleep(0.01)
    conn.close()
    os._exit(0)


# -- full-size multi-process runs (BASELINE configs[3-4]: 1B / 7B bf16) -------------------------
# Parameters and training deltas are closed-form functions of the element index, computed the
# same way on the device (chunked, int64 torch ops) and in numpy for a few sampled windows, so
# the oracle replays the windows without materialising 7B elements on the host.  Values are
# k / 2^23 - 1/2 with an integer k < 2^23 (exact in fp32), deltas the same times 2^-7.
_CHUNK = 1 << 27


def synth_f32(idx, g, r):
    """fp32 values at int64 indices `idx` for rank g; r = -1: initial parameters, r >= 0: the
    training delta of round r.  Works on numpy arrays and on torch tensors alike."""
    m = (1 << 23) - 1        # the low and high index bits hashed apart: no int64 overflow
    k = ((idx & m) * 5039617 + (idx >> 23) * 3141597 + (g * 40503 + (r + 1) * 977)) & m
    if isinstance(k, np.ndarray):
        v = k.astype(np.float32) * np.float32(2.0 ** -23) - np.float32(0.5)
        return v * np.float32(2.0 ** -7) if r >= 0 else v
    import torch
    v = k.to(torch.float32) * (2.0 ** -23) - 0.5
    return v * (2.0 ** -7) if r >= 0 else v


def synth_windows(n):
    """Sampled [begin, end) windows: head, middle, a ragged tail."""
    return [(0, 4096), (n // 2 - 2048, n // 2 + 2048), (n - 4099, n)]


def synth_losses(world, T):
    """Losses crossing a 0.5 divergence threshold within T rounds (configs[3])."""
    send = [[1.2 * 0.55 ** r + 0.01 * g for g in range(world)] for r in range(T)]
    wait = [[1.1 * 0.55 ** r + 0.02 * g for g in range(world)] for r in range(T)]
    return send, wait


def _synth_fill(flat, g, r, add):
    import torch
    n = flat.numel()
    for b in range(0, n, _CHUNK):
        e = min(n, b + _CHUNK)
        v = synth_f32(torch.arange(b, e, device=flat.device, dtype=torch.int64), g, r).to(flat.dtype)
        if add:
            flat[b:e].add_(v)
        else:
            flat[b:e].copy_(v)


def big_worker(rank, world, port, cfg_path, out_dir, n, T, pull, dtype):
    """Lock-step rounds at full size (DistGroup over IPC, gloo barrier on one GPU); records the
    sampled windows of the parameters after every round, the clocks and the peers."""
    import time
    t0 = time.perf_counter()

    def log(msg):
        sys.stderr.write("[big_worker r%d +%.1fs] %s\n" % (rank, time.perf_counter() - t0, msg))
        sys.stderr.flush()
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    log("process group up")
    from dpwa_amd import DpwaConnection
    names = ["r%d" % i for i in range(world)]
    conn = DpwaConnection(names[rank], cfg_path, seed=500 + rank, pull=pull, group="lockstep")
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    flat = torch.empty(n, dtype=tdt, device=dev)
    _synth_fill(flat, rank, -1, add=False)
    torch.cuda.synchronize()
    log("%d parameters filled" % n)
    send, wait = synth_losses(world, T)
    wins, clocks, peers = [], np.zeros(T), []
    trace = os.environ.get("DPWA_TEST_TRACE") == "1"

    def step(msg):
        if trace:
            torch.cuda.synchronize()
            log(msg)
    for r in range(T):
        conn.update_send(flat, send[r][rank], reuse_snapshot=r >= 2)
        step("round %d: update_send" % r)
        _synth_fill(flat, rank, r, add=True)
        step("round %d: training step" % r)
        if r == 0:
            payload, _ = conn.update_wait(wait[r][rank])
            step("round %d: update_wait" % r)
            if payload is not None:
                conn.average(flat)
        else:                           # the adapter's default: fused, write-through
            payload, _ = conn.update_wait_average(flat, wait[r][rank], write_through=True)
        step("round %d: averaged" % r)
        peers.append(payload.peer if payload is not None else "")
        wins.append(np.concatenate([to_host(flat[b:e]) for b, e in synth_windows(n)]))
        clocks[r] = conn.clock
        log("round %d done (peer %s)" % (r, peers[-1] or "-"))
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), params=np.stack(wins), clocks=clocks, peers=np.array(peers))
    torch.cuda.synchronize()
    dist.barrier()
    conn.close()
    dist.destroy_process_group()


def resnet_worker(rank, world, port, cfg_path, out_dir, T, group):
    """The reference's training loop (examples/pytorch-cifar/main.py:122-158) on one rank:
    CIFAR ResNet-18, synthetic batches, SGD, the adapter's parameters gossiped every step over
    the multi-process group.  update_wait goes through the connection seam (payload, factor),
    so the fetched snapshot can be recorded before the reference's lerp is applied.  Records
    per round the sha1 of the snapshot it published and of the one it fetched, the peer, the
    clock, the losses, and whether the average equals oracle.lerp(before, fetched, factor)."""
    import hashlib
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    from resnet18_gossip import resnet18

    from dpwa_amd import DpwaPyTorchAdapter
    from oracle.lerp import bits_equal, lerp_f32
    names = ["w%d" % (i + 1) for i in range(world)]
    torch.manual_seed(rank)
    net = resnet18().to(dev)
    adapter = DpwaPyTorchAdapter(net, names[rank], cfg_path, seed=100 + rank, group=group)
    conn, flat = adapter.connection, adapter.flat.buffer
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    gen = torch.Generator(device=dev).manual_seed(5 + rank)

    def sha(t):
        return hashlib.sha1(t.cpu().numpy().tobytes()).hexdigest()
    rec = {k: [] for k in ("published", "fetched", "peers", "clocks", "send", "wait", "ok")}
    send = 2.3
    for r in range(T):
        adapter.update_send(send)
        rec["published"].append(sha(flat))
        x = torch.randn(8, 3, 32, 32, device=dev, generator=gen)
        y = torch.randint(0, 10, (8,), device=dev, generator=gen)
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(net(x), y)
        loss.backward()
        opt.step()
        wait = float(loss)
        before = flat.cpu().numpy()
        payload, factor = conn.update_wait(wait)
        if payload is None:
            rec["fetched"].append("")
            rec["peers"].append("")
            rec["ok"].append(bits_equal(flat.cpu().numpy(), before))
        else:
            snap = payload.tensor()
            rec["fetched"].append(sha(snap))
            rec["peers"].append(payload.peer)
            f = float(factor)
            conn.average(flat)
            rec["ok"].append(bits_equal(flat.cpu().numpy(), lerp_f32(before, snap.cpu().numpy(), f)))
        rec["clocks"].append(conn.clock)
        rec["send"].append(send)
        rec["wait"].append(wait)
        send = wait
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), **{k: np.array(v) for k, v in rec.items()})
    torch.cuda.synchronize()
    dist.barrier()
    conn.close()
    dist.destroy_process_group()


def async_timeout_worker(rank, world, port, cfg_path, out_dir, n, T, hold_round, pull="copy"):
    """Free-running rounds (the gossip board) where rank 0's pull of round `hold_round` is held
    on its side stream behind a spin kernel (tests.helpers.Hold: HOLD_S from the measured spin
    rate) and its update_wait comes HOST_WAIT_S later, past the config's timeout_ms (TIMEOUT_MS):
    that request times out (conn.py:304-309), the loop picks again and the re-selected pull goes
    to a rescue lane.  Records what async_worker records plus the fetch attempts and scores."""
    import ctypes
    import time
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dpwa_amd import DpwaConnection, _lib
    from tests.helpers import HOST_WAIT_S, Hold
    names = ["r%d" % i for i in range(world)]
    conn = DpwaConnection(names[rank], cfg_path, seed=710 + rank, group="async", pull=pull)
    flat = torch.empty(n, device=dev, dtype=torch.float32)
    bases = [torch.from_numpy(async_base(rank, r, n)).to(dev) for r in range(T)]
    params, clocks, peers, versions, scores, attempts = np.zeros((T, n), np.float32), np.zeros(T), [], [], [], []
    for r in range(T):
        flat.copy_(bases[r])
        held = None
        if rank == 0 and r == hold_round:
            s = ctypes.c_void_p()
            _lib.call("dpwa_learner_side_stream", conn._learner.handle, ctypes.byref(s))
            held = Hold(torch.cuda.ExternalStream(s.value, device=dev))   # this round's pull queues behind it
        conn.update_send(flat, async_loss(rank, r))
        if held:
            time.sleep(HOST_WAIT_S)                     # past timeout_ms
        payload, _ = conn.update_wait_average(flat, async_loss(rank, r, wait=True))
        peers.append(payload.peer if payload is not None else "")
        versions.append(conn._info()[2] if payload is not None else 0)
        attempts.append(conn.last_fetch_attempts)
        params[r] = flat.cpu().numpy()
        clocks[r] = conn.clock
        scores.append([conn.flow_control_scores()[p] for p in names if p != names[rank]])
        if held:
            torch.cuda.synchronize()                    # the stalled pull has landed
            held.check(HOST_WAIT_S)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), params=params, clocks=clocks, peers=np.array(peers),
             versions=np.array(versions, dtype=np.int64), attempts=np.array(attempts),
             scores=np.array([[-1 if s is None else s for s in row] for row in scores]))
    dist.barrier()
    conn.close()
    dist.destroy_process_group()
