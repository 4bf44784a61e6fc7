"""Free-running gossip between processes (AsyncDistGroup + the gossip board) on the GPU box:
ranks share the one GPU, map each other's snapshot slots over IPC and never wait for each
other.  Which version of a peer a round reads depends on timing, so the check is
consistency with the reference's semantics rather than one fixed trajectory: every average
equals the oracle lerp of this round's parameters with exactly the snapshot version the
board handed out (a torn or overwritten snapshot would not), versions never go backwards,
the clocks follow dpwa.py:155 through those versions, and a rank that dies mid-run reads
as a refused connection (conn.py:253-256) instead of stalling anyone."""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle.async_check import AsyncRuns
from tests import dist_worker

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def check_run(tmp_path, world, n, T, ranks, interp="constant", thr=0.0):
    names = ["r%d" % i for i in range(world)]
    runs = {g: np.load(tmp_path / ("rank%d.npz" % g)) for g in ranks}
    check = AsyncRuns(names, {g: runs[g]["peers"] for g in ranks}, {g: runs[g]["versions"] for g in ranks},
                      interp, 0.5, thr)
    averaged = 0
    for g in ranks:
        bad = check.check_rank(g, runs[g]["params"], runs[g]["clocks"], n)
        assert not bad, (g, bad[:5])
        averaged += sum(1 for p in runs[g]["peers"] if str(p) != "")
    return runs, averaged


def empty_rounds_form_a_prefix(run):
    """With fetch_probability 1 a round reads nothing only while every peer still has no
    publish (the empty replies of conn.py:301-302 send TxThread back to pick again until a
    peer with state answers).  A peer's version never returns to 0 while it lives, so once
    any round has averaged, every later round must too: the empty rounds are a prefix."""
    peers = [str(p) for p in run["peers"]]
    k = next((i for i, p in enumerate(peers) if p != ""), len(peers))
    return all(p != "" for p in peers[k:]), k


@pytest.mark.parametrize("world,pull,interp,fp,thr", [(2, "copy", "constant", 1.0, 0.0),
                                                      (3, "kernel:64", "constant", 1.0, 0.0),
                                                      (3, "copy", "clock", 1.0, 0.0),
                                                      (3, "kernel", "loss", 0.7, 0.5)])
def test_async_gossip_reads_whole_snapshots(tmp_path, world, pull, interp, fp, thr):
    n, T = 1_000_003, 40
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "async.yaml")
    dist_worker.write_cfg(cfg, names, fp, interp, thr)
    mp.spawn(dist_worker.async_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, pull), nprocs=world,
             join=True)
    runs, averaged = check_run(tmp_path, world, n, T, range(world), interp, thr)
    if fp == 1.0:
        for g in range(world):
            prefix, k = empty_rounds_form_a_prefix(runs[g])
            assert prefix and k < T, (g, [str(p) for p in runs[g]["peers"]])
    else:
        assert averaged >= world * T * fp * 0.5


def test_async_gossip_survives_a_rank_that_leaves(tmp_path):
    """r2 leaves the board at its round 5 and exits without any teardown: the others finish
    every round, never read past its last publish, and score it down as refused
    (conn.py:253-256, 270-272).  (A killed process reads the same way through its dead pid:
    tests/test_board.py.)"""
    world, n, T, die = 3, 200_003, 30, 5
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "dead.yaml")
    dist_worker.write_cfg(cfg, names, 1.0, "constant", 0.0)
    mp.spawn(dist_worker.async_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, "copy", 2, die),
             nprocs=world, join=True)
    runs, _ = check_run(tmp_path, world, n, T, [0, 1])
    for g in (0, 1):
        run = runs[g]
        read_r2 = [int(v) for p, v in zip(run["peers"], run["versions"]) if str(p) == "r2"]
        assert all(v <= die for v in read_r2), read_r2
        assert run["scores"][-1][1] < 1000, run["scores"][-1]      # r2 is the second peer of r0 and r1


@pytest.mark.parametrize("world,pull,interp", [(2, "copy", "constant"), (3, "kernel:64", "clock")])
def test_async_write_through_snapshots(tmp_path, world, pull, interp):
    """Write-through under the board: the averaging kernel writes the next snapshot (and, for
    constant/clock interpolation, its header), the publish moves no bytes, and the publish
    rule still holds -- no reader ever averages a snapshot other than exactly what the
    publisher had at that publish (reconstructed from the publisher's own recorded results)."""
    n, T = 500_003, 30
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "async_wt.yaml")
    dist_worker.write_cfg(cfg, names, 1.0, interp, 0.0)
    mp.spawn(dist_worker.async_wt_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, pull), nprocs=world,
             join=True)
    runs = {g: np.load(tmp_path / ("rank%d.npz" % g)) for g in range(world)}

    def published(q, v, n_):
        from oracle.async_check import async_base
        return async_base(q, -1, n_) if v == 1 else runs[q]["params"][v - 2]

    check = AsyncRuns(names, {g: runs[g]["peers"] for g in range(world)},
                      {g: runs[g]["versions"] for g in range(world)}, interp, 0.5, 0.0, published=published)
    for g in range(world):
        bad = check.check_rank(g, runs[g]["params"], runs[g]["clocks"], n)
        assert not bad, (g, bad[:5])
        prefix, k = empty_rounds_form_a_prefix(runs[g])
        assert prefix and k < T


def test_async_write_through_bf16(tmp_path):
    """bf16 (BASELINE configs[3-4]'s dtype) through the free-running board with write-through
    snapshots: every average against the oracle's torch-eager bf16 lerp of the exact snapshot
    version read, clocks exact."""
    from oracle.async_check import async_base_bf16
    from oracle.lerp import lerp_bf16
    world, n, T, interp = 3, 300_007, 24, "clock"
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "async_bf16.yaml")
    dist_worker.write_cfg(cfg, names, 1.0, interp, 0.0)
    mp.spawn(dist_worker.async_wt_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, "kernel:64", "bf16"),
             nprocs=world, join=True)
    runs = {g: np.load(tmp_path / ("rank%d.npz" % g)) for g in range(world)}

    def published(q, v, n_):
        return async_base_bf16(q, -1, n_) if v == 1 else runs[q]["params"][v - 2]

    check = AsyncRuns(names, {g: runs[g]["peers"] for g in range(world)},
                      {g: runs[g]["versions"] for g in range(world)}, interp, 0.5, 0.0, published=published,
                      base=async_base_bf16, lerp=lerp_bf16)
    for g in range(world):
        bad = check.check_rank(g, runs[g]["params"], runs[g]["clocks"], n)
        assert not bad, (g, bad[:5])


def test_async_write_through_vmm_shared_slots(tmp_path, monkeypatch):
    """The free-running board over fd-shared (hipMemCreate) snapshot slots, DPWA_VMM=1."""
    monkeypatch.setenv("DPWA_VMM", "1")
    test_async_write_through_snapshots(tmp_path, 3, "copy", "clock")
