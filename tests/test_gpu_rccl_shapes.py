"""The RCCL (`nccl` backend) code shapes of the multi-GPU groups, on one GPU.

RCCL refuses two ranks on one device, so the multi-process GPU tests run over gloo and the
`nccl` branches of dpwa_amd/group.py would otherwise first execute in the driver's 8-GPU run.
A world-size-1 RCCL group runs every one of those call shapes -- dtype, device, the stream they
are ordered on -- so argument and stream mistakes surface here:
  * DistGroup.barrier: the stream-ordered all_reduce of the lock-step round (after_publish),
    through the real API (a one-node config: publishes, gates, no peer);
  * DistGroup._exchange_picks: the all_gather_into_tensor of the relay's picks;
  * DistGroup._side_barrier: the all_reduce on the learner's side stream between relay phases;
  * the object all-gathers of on_bind / _single_host, and bench.py's gloo control group beside
    an RCCL default group.
What only a multi-GPU run can show -- the collectives actually exchanging data between
devices, cross-device IPC mappings and the system-scope L2 fences -- is listed in DESIGN.md §6."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, cfg, out):
    import json
    import torch.distributed as dist
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from dpwa_amd import DpwaConnection
    from dpwa_amd.group import DistGroup
    res = {}
    conn = DpwaConnection("solo", cfg, seed=1, group="lockstep")
    g = conn._group
    res["group"] = type(g).__name__
    res["backend"] = g.backend
    flat = torch.randn(4099, device=dev)
    before = flat.clone()
    for _ in range(3):                       # publish -> RCCL barrier on the stream -> gate
        conn.update_send(flat, 1.0)
        payload, factor = conn.update_wait_average(flat, 1.0)
        res.setdefault("payloads", []).append(payload is None and factor == 0)
    res["clock"] = conn.clock                # clock += 1 per publish, no averaging
    res["unchanged"] = bool(torch.equal(flat, before))
    res["flag"] = int(g._flag.item())
    assert isinstance(g, DistGroup)
    # the relay's collectives, with the tensors on_bind would give them
    g._pick = torch.full((1,), -1, dtype=torch.int32, device=dev)
    g._picks = torch.full((1,), -5, dtype=torch.int32, device=dev)
    g._side = torch.cuda.Stream(dev)
    torch.cuda._sleep(20_000_000)            # the exchange is ordered after this on the stream
    g._exchange_picks(7, dev)
    g._side_barrier(dev)
    torch.cuda.synchronize()
    res["picks"] = g._picks.tolist()
    res["flag_side"] = int(g._flag_side.item())
    # bench.py's control plane: a gloo group beside the RCCL default group
    import bench
    ctl = dist.new_group(backend="gloo")
    res["agree"] = bench._agree(True, 1, ctl)
    got = [None]
    dist.all_gather_object(got, {"x": 1}, group=ctl)
    res["ctl_gather"] = got
    conn.close()
    dist.destroy_process_group()
    with open(out, "w") as f:
        json.dump(res, f)


def test_rccl_code_shapes_world_one(tmp_path):
    cfg = tmp_path / "solo.yaml"
    cfg.write_text("- nodes:\n  - {name: solo, host: 127.0.0.1, port: 45999}\n- fetch_probability: 1\n"
                   "- timeout_ms: 2500\n- interpolation: clock\n- divergence_threshold: 0\n"
                   "- constant: { value: 0.5 }\n- clock: 0\n- loss: 0\n")
    out = tmp_path / "res.json"
    mp.spawn(_worker, args=(_free_port(), str(cfg), str(out)), nprocs=1, join=True)
    import json
    res = json.loads(out.read_text())
    assert res["group"] == "DistGroup" and res["backend"] == "nccl"
    assert res["payloads"] == [True, True, True]
    assert res["clock"] == 3.0 and res["unchanged"]
    assert res["flag"] == 0 and res["flag_side"] == 0
    assert res["picks"] == [7]
    assert res["agree"] is True and res["ctl_gather"] == [{"x": 1}]
