"""Gossip-state checkpoint (extension; SURVEY §5 checkpoint/resume): the reference keeps no
gossip state across a restart (dpwa.py:59 starts the clock at 0, `random` starts from its seed).
DpwaConnection.state_dict() / load_state_dict() carry the clock and the scheduler (generator,
flow-control scores, peer order).  CPU: the connection-level round trip of the scheduler and the
validation; the GPU test (test_gpu_gossip.py) resumes a gossip mid-run against the uninterrupted one."""
import json

import pytest

from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter  # noqa: F401
from dpwa_amd.group import LocalGroup


def _cfg(path, names, fp=0.7):
    lines = ["- nodes:"] + ["  - {name: %s, host: localhost, port: %d}" % (n, 47100 + i) for i, n in enumerate(names)]
    lines += ["- fetch_probability: %r" % fp, "- timeout_ms: 2500", "- interpolation: clock",
              "- divergence_threshold: 0", "- constant: 0", "- clock: 0", "- loss: 0"]
    path.write_text("\n".join(lines) + "\n")


def test_connection_state_round_trips_through_json(tmp_path):
    names = ["a", "b", "c", "d"]
    cfg = tmp_path / "c.yaml"
    _cfg(cfg, names)
    a = DpwaConnection("b", str(cfg), seed=11, group=LocalGroup())
    for _ in range(25):                       # gate draws, picks and flow control without a GPU
        a._sched.bernoulli()
        a._sched.fetch([0, 3, 1])
    state = json.loads(json.dumps(a.state_dict()))     # plain data
    assert state["name"] == "b" and state["peers"] == ["a", "c", "d"] and state["clock"] == 0.0
    b = DpwaConnection("b", str(cfg), seed=999, group=LocalGroup())
    b.load_state_dict(state)
    assert b._sched.get_state() == a._sched.get_state()
    assert b.flow_control_scores() == a.flow_control_scores()
    assert [a._sched.fetch([0, 0, 2]) for _ in range(20)] == [b._sched.fetch([0, 0, 2]) for _ in range(20)]
    state["clock"] = 41.0
    b.load_state_dict(state)                  # before the first round: written at bind
    assert b.state_dict()["clock"] == 41.0
    a.close()
    b.close()


def test_state_of_another_node_is_refused(tmp_path):
    names = ["a", "b", "c"]
    cfg = tmp_path / "c.yaml"
    _cfg(cfg, names)
    a = DpwaConnection("a", str(cfg), seed=1, group=LocalGroup())
    b = DpwaConnection("b", str(cfg), seed=1, group=LocalGroup())
    with pytest.raises(ValueError, match="does not fit"):
        b.load_state_dict(a.state_dict())
    with pytest.raises(ValueError, match="format"):
        b.load_state_dict({"format": 0})
    a.close()
    b.close()


def test_state_goes_through_torch_save_and_the_safe_loader(tmp_path):
    """The INTEGRATION recipe: torch.save beside the model, torch.load(weights_only=True)."""
    import torch
    names = ["a", "b", "c"]
    cfg = tmp_path / "c.yaml"
    _cfg(cfg, names)
    a = DpwaConnection("c", str(cfg), seed=5, group=LocalGroup())
    for _ in range(9):
        a._sched.fetch([0, 1])
    torch.save({"gossip": a.state_dict()}, tmp_path / "ck.pt")
    st = torch.load(tmp_path / "ck.pt", weights_only=True)["gossip"]
    b = DpwaConnection("c", str(cfg), seed=6, group=LocalGroup())
    b.load_state_dict(st)
    assert b._sched.get_state() == a._sched.get_state()
    a.close()
    b.close()
