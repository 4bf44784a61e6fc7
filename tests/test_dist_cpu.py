"""Multi-process control plane on the CPU (gloo, world size 2, 3 and 8 -- the full-node rank count): every rank builds its
DpwaConnection exactly as under torchrun, gets the DistGroup, maps node index <-> rank,
and its native scheduler drives lock-step rounds whose Bernoulli draws and peer choices
must equal the oracle's (CPython random, dpwa/conn.py:224-317).  The data path needs a
GPU and is covered by tests/test_gpu_ipc.py."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from tests import dist_worker


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def control_worker(rank, world, port, cfg, out_dir, T):
    import json

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dpwa_amd import DpwaConnection, _lib
    from dpwa_amd.group import AsyncDistGroup, DistGroup
    names = ["r%d" % i for i in range(world)]
    conn = DpwaConnection(names[rank], cfg, seed=500 + rank)
    assert isinstance(conn._group, AsyncDistGroup)      # free-running rounds by default
    lock = DpwaConnection(names[rank], cfg, seed=500 + rank, group="lockstep")
    assert type(lock._group) is DistGroup
    lock.close()
    assert conn._group.rank == rank
    assert [conn.peer_rank(k) for k in range(len(conn.peers))] == [r for r in range(world) if r != rank]
    err = None
    try:
        DistGroup(conn.nodes, names[(rank + 1) % world])
    except ValueError as e:
        err = str(e)
    assert err and "rank %d" % rank in err
    trace = []
    ready = [_lib.PEER_READY] * len(conn.peers)
    for r in range(T):
        fetching = conn._sched.bernoulli()
        peer = None
        if fetching:
            k, attempts = conn._sched.fetch(ready)
            assert attempts == 1
            peer = conn.peers[k].name
        trace.append(peer)
    traces = [None] * world
    dist.all_gather_object(traces, trace)
    if rank == 0:
        with open(os.path.join(out_dir, "traces.json"), "w") as f:
            json.dump(traces, f)
    conn.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fp", [(2, 1.0), (3, 0.7), (8, 0.7)])
def test_dist_control_plane_matches_oracle(tmp_path, world, fp):
    import json

    from oracle.policy import OracleLearner
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "d.yaml")
    dist_worker.write_cfg(cfg, names, fp, "clock", 0.0)
    T = 60
    mp.spawn(control_worker, args=(world, free_port(), cfg, str(tmp_path), T), nprocs=world, join=True)
    traces = json.load(open(tmp_path / "traces.json"))
    for r in range(world):
        L = OracleLearner(names[r], [n for n in names if n != names[r]], fp, "clock", None, 0.0, 500 + r)
        want = []
        for _ in range(T):
            L.update_send(1.0)
            if L.fetching:
                _, _, att = L.fetch(lambda p: "ok", lambda p: ("payload", {}, b"x"))
                want.append(att[-1]["peer"])
            else:
                want.append(None)
        assert traces[r] == want, r


def multihost_worker(rank, world, port, cfg):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # what torchrun exports for a job of `world` ranks spread one per host
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_WORLD_SIZE"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dpwa_amd import DpwaConnection
    try:
        DpwaConnection("r%d" % rank, cfg, seed=1)
    except ValueError as e:
        assert "several hosts" in str(e) and "transport='wire'" in str(e), e
    else:
        raise AssertionError("a multi-host job must not get the IPC/xGMI group")
    dist.barrier()
    dist.destroy_process_group()


def test_multi_host_job_is_refused_the_ipc_group(tmp_path):
    """A torchrun job spanning hosts cannot map peers' HBM: it gets a clear error naming the
    wire transport instead of a hipIpcOpenMemHandle failure at the first publish."""
    cfg = str(tmp_path / "mh.yaml")
    dist_worker.write_cfg(cfg, ["r0", "r1"], 1.0, "constant", 0.0)
    mp.spawn(multihost_worker, args=(2, free_port(), cfg), nprocs=2, join=True)
