"""Multi-process gossip through the production DistGroup path on the GPU box: two ranks
share the one GPU, map each other's snapshot slots with hipIpcOpenMemHandle and pull them
on their side streams, lock-step, checked against the oracle simulation.  (RCCL refuses
two ranks on one device, so the barrier runs over gloo here; the data path -- IPC-mapped
slots, side-stream pulls, device factor, fused lerp -- is the production one.)"""
import functools
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
                                                       (3, "clock", 0.7, 0.0, "kernel")])
def test_ipc_gossip_matches_oracle(tmp_path, world, interp, fp, thr, pull):
    n, T = 100_003, 12
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "dist.yaml")
    dist_worker.write_cfg(cfg, names, fp, interp, thr)
    mp.spawn(dist_worker.gossip_worker, args=(world, free_port(), cfg, str(tmp_path), n, T, "gloo", 0, pull),
             nprocs=world, join=True)
    init, deltas, send, wait = dist_worker.inputs(world, n, T)
    exp = ogossip.simulate(names, init, deltas, send, wait, interp, 0.5, thr, fp, [500 + r for r in range(world)])
    for r in range(world):
        got = np.load(tmp_path / ("rank%d.npz" % r))
        want_peers = [p[0] if p else "" for p in (exp["picks"][t][r] for t in range(T))]
        assert list(got["peers"]) == want_peers, r
        assert np.array_equal(got["clocks"], exp["clocks"][:, r]), r
        assert olerp.bits_equal(got["params"], exp["params"][:, r]), r
