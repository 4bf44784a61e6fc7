"""bench.py's parity leg (the self-check the driver's multi-GPU bench runs after its timed
region) on the GPU box:

* on one GPU: two ranks on the same device over gloo, through every transport the bench's
  N>1 trials use (lock-step copy / kernel / relay pulls and free-running board rounds), so the
  leg itself is known to pass before the driver's 8-GPU run relies on it;
* across real devices (RCCL, one rank per GPU, cross-device IPC, the system-scope L2
  coherence kernels and the RCCL stream-ordered barrier) when the box has more than one GPU;
  skipped otherwise."""
import os
import socket
import sys
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

TRANSPORTS = ["lockstep/copy", "lockstep/kernel:256", "lockstep/relay:32", "lockstep/relay-avg:32", "async/copy",
              "async/kernel:256", "async/copy+wt", "async/kernel:256+wt"]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def parity_worker(rank, world, port, backend, per_device, out_dir):
    import json
    import torch.distributed as dist
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", rank if per_device else 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    with tempfile.TemporaryDirectory() as tmp:
        res = bench.parity_leg(world, rank, rank, dev, tmp, TRANSPORTS, backend)
    if rank == 0:
        with open(os.path.join(out_dir, "parity.json"), "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, world, backend, per_device):
    import json
    mp.spawn(parity_worker, args=(world, free_port(), backend, per_device, str(tmp_path)), nprocs=world, join=True)
    res = json.load(open(tmp_path / "parity.json"))
    assert res == {t: True for t in TRANSPORTS}, res


def test_parity_leg_two_ranks_one_gpu(tmp_path):
    _run(tmp_path, 2, "gloo", False)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs more than one GPU (cross-device IPC over xGMI)")
def test_parity_leg_across_devices(tmp_path):
    _run(tmp_path, min(torch.cuda.device_count(), 4), "nccl", True)


def test_parity_leg_local_one_process():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    with tempfile.TemporaryDirectory() as tmp:
        res = bench.parity_leg(1, 0, 0, torch.device("cuda", 0), tmp, ["self", "local"], "nccl")
    assert res == {"self": True, "local": True}
