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

from oracle import lerp as olerp
from oracle.policy import factor_and_clock
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
    c_after = {}

    def policy(g, r):           # dpwa.py:143-155 for rank g's round r against what it read
        q, v = names.index(str(runs[g]["peers"][r])), int(runs[g]["versions"][r])
        return factor_and_clock(interp, 0.5, thr, c_pub(g, r), c_pub(q, v - 1), dist_worker.async_loss(g, r, True),
                                dist_worker.async_loss(q, v - 1))

    def c_pub(g, r):            # the clock rank g published at its round r (dpwa.py:112)
        return (c_after_of(g, r - 1) if r > 0 else 0.0) + 1.0

    def c_after_of(g, r):       # its clock after that round's update_wait (dpwa.py:155)
        if (g, r) not in c_after:
            run = runs[g]
            if run["peers"][r] == "":
                c_after[(g, r)] = c_pub(g, r)
            else:
                c_after[(g, r)] = policy(g, r)[1]
        return c_after[(g, r)]

    averaged = 0
    for g in ranks:
        run = runs[g]
        last = {}
        for r in range(T):
            mine = dist_worker.async_base(g, r, n)
            peer = str(run["peers"][r])
            if peer == "":
                want = mine
            else:
                q, v = names.index(peer), int(run["versions"][r])
                assert 1 <= v, (g, r)
                assert v >= last.get(q, 0), (g, r, "versions went backwards")
                last[q] = v
                if len(runs) == world:
                    factor = policy(g, r)[0]
                else:           # a rank's clocks are unknown once it has gone: constant only
                    assert interp == "constant" and thr == 0.0
                    factor = 0.5
                want = olerp.lerp_f32(mine, dist_worker.async_base(q, v - 1, n), factor)
                averaged += 1
            assert olerp.bits_equal(run["params"][r], want), (g, r, peer)
            if all(q in runs for q in range(world)):
                assert run["clocks"][r] == c_after_of(g, r), (g, r)
    return runs, averaged


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
    _, averaged = check_run(tmp_path, world, n, T, range(world), interp, thr)
    if fp == 1.0:
        assert averaged >= world * (T - 5)     # only rounds before the peers' first publishes may be empty
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
