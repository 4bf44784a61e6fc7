"""DpwaConfiguration / DpwaConnection construction against the reference's own parse of
the same YAML documents (tests/golden/config.json).  CPU only: no learner is created
before the first update_send."""
import pytest

from dpwa_amd import DpwaConfiguration, DpwaConnection
from dpwa_amd.group import LocalGroup
from dpwa_amd.interpolation import ClockWeightedInterpolation
from tests.helpers import load_json


@pytest.fixture
def cfgfiles(tmp_path):
    data = load_json("config.json")["files"]
    paths = {}
    for name, rec in data.items():
        p = tmp_path / (name.strip("_") + ("" if name.endswith(".yaml") else ".yaml"))
        p.write_text(rec["text"])
        paths[name] = (str(p), rec)
    return paths


def test_configuration_matches_reference(cfgfiles):
    for name, (path, rec) in cfgfiles.items():
        if name.startswith("_"):
            continue
        c = DpwaConfiguration(path)
        assert c.config == rec["config"]
        assert c.get_nodes() == rec["nodes"]
        assert list(c.get_interpolation()) == rec["interpolation"]
        assert c.get_timeoutms() == rec["timeout_ms"]
        assert c.get_fetch_probability() == rec["fetch_probability"]
        assert c.get_divergence_threshold() == rec["divergence_threshold"]


def test_connection_fields_match_reference(cfgfiles):
    for name, (path, rec) in cfgfiles.items():
        if name.startswith("_"):
            continue
        for node, conn_rec in rec["connections"].items():
            conn = DpwaConnection(node, path, seed=0, group=LocalGroup())
            assert conn.me.__dict__ == conn_rec["me"]
            assert [p.__dict__ for p in conn.peers] == conn_rec["peers"]
            assert type(conn.interpolation).__name__ == conn_rec["interp_class"]
            assert conn.divergence_threshold == conn_rec["divergence_threshold"]
            assert conn.clock == conn_rec["clock"]
            assert conn.fetching is False
            assert list(conn.flow_control_scores().values()) == [1000] * len(conn.peers)


def test_bad_constant_raises_like_reference(cfgfiles):
    path, rec = cfgfiles["_bad_constant"]
    assert rec["raises"] == "AssertionError"
    with pytest.raises(AssertionError):
        DpwaConnection("w1", path, group=LocalGroup())


def test_bad_method_raises_like_reference(cfgfiles):
    path, rec = cfgfiles["_bad_method"]
    assert rec["raises"] == "KeyError"
    with pytest.raises(KeyError):
        DpwaConnection("w1", path, group=LocalGroup())


def test_unknown_node_raises(cfgfiles):
    path, _ = cfgfiles["four_nodes.yaml"]
    with pytest.raises(AttributeError):
        DpwaConnection("nope", path, group=LocalGroup())


def test_duplicate_node_in_process_is_refused(cfgfiles):
    path, _ = cfgfiles["four_nodes.yaml"]
    g = LocalGroup()
    a = DpwaConnection("w1", path, group=g)
    with pytest.raises(OSError):
        DpwaConnection("w1", path, group=g)
    a.close()
    DpwaConnection("w1", path, group=g)


def test_seed_extension(tmp_path):
    p = tmp_path / "s.yaml"
    p.write_text("- nodes:\n  - {name: a, host: h, port: 1, seed: 17}\n  - {name: b, host: h, port: 2}\n"
                 "- seed: 99\n- fetch_probability: 0.5\n- timeout_ms: 1\n- interpolation: clock\n- clock: 0\n"
                 "- divergence_threshold: 0\n")
    c = DpwaConfiguration(str(p))
    assert c.get_seed("a") == 17 and c.get_seed("b") == 99
    conn = DpwaConnection("b", str(p), group=LocalGroup())
    assert isinstance(conn.interpolation, ClockWeightedInterpolation)
    import random
    r = random.Random(99)
    assert [conn._sched.bernoulli() for _ in range(20)] == [r.random() < 0.5 for _ in range(20)]


def test_interpolation_host_formulas():
    from dpwa_amd.interpolation import ConstantInterpolation, LossInterpolation
    assert ConstantInterpolation(0.25)(1, 2, 3, 4) == 0.25
    assert ClockWeightedInterpolation()(1, 3, 0, 0) == 0.75
    assert LossInterpolation()(1.0, 3.0, 1.0, 3.0) == 0.25
    with pytest.raises(ZeroDivisionError):
        LossInterpolation()(0, 0, 0.0, 0.0)


def test_launch_make_config_roundtrip(tmp_path):
    from dpwa_amd.launch import main, write_config
    out = tmp_path / "gen.yaml"
    assert main(["make-config", "--nodes", "8", "--out", str(out), "--interpolation", "clock", "--seed", "7"]) == 0
    c = DpwaConfiguration(str(out))
    assert [n["name"] for n in c.get_nodes()] == ["w%d" % i for i in range(1, 9)]
    assert c.get_interpolation() == ("clock", 0) and c.get_fetch_probability() == 1 and c.get_seed("w3") == 7
    conn = DpwaConnection("w3", str(out), group=LocalGroup())
    assert [p.name for p in conn.peers] == ["w1", "w2", "w4", "w5", "w6", "w7", "w8"]
    with pytest.raises(ValueError):
        write_config(str(tmp_path / "x.yaml"), ["a"], interpolation="cubic")


def test_reference_loads_generated_config(tmp_path):
    """What dpwa_amd.launch writes -- the reference schema plus the per-node gpu: key -- is
    what the reference itself parsed into tests/golden/config.json (launch_*.yaml entries,
    made by tests/golden/make_golden.py through the reference's DpwaConfiguration and
    DpwaConnection): the same text, and our parse equals the reference's."""
    from dpwa_amd.launch import config_text
    files = load_json("config.json")["files"]
    assert config_text(["w0", "w1", "w2"], gpus=[0, 1, 2], interpolation="clock",
                       divergence_threshold=0.5) == files["launch_gpu.yaml"]["text"]
    assert config_text(["w1", "w2"], fetch_probability=0.7, interpolation="loss") == files["launch_plain.yaml"]["text"]
    rec = files["launch_gpu.yaml"]
    assert [n["gpu"] for n in rec["nodes"]] == [0, 1, 2]
    assert rec["connections"]["w2"]["me"] == {"name": "w2", "host": "localhost", "port": 45002, "gpu": 2}
    p = tmp_path / "g.yaml"
    p.write_text(rec["text"])
    c = DpwaConfiguration(str(p))
    assert c.config == rec["config"]
    assert [c.get_gpu(n) for n in ("w0", "w1", "w2")] == [0, 1, 2]


def test_prepare_writes_config_and_torchrun_script(tmp_path):
    """prepare.py:17-40 for a GPU node: one node per GPU with its gpu: key, and a run.sh that
    starts one rank per GPU; rank r finds node r and its device."""
    import os
    import stat
    from dpwa_amd.launch import main, node_for_rank
    assert main(["prepare", "--gpus", "4", "--out-dir", str(tmp_path), "--script", "main.py",
                 "--interpolation", "clock", "--", "--lr=0.01", "--batch-size", "8"]) == 0
    cfg = tmp_path / "dpwa.yaml"
    c = DpwaConfiguration(str(cfg))
    assert [n["name"] for n in c.get_nodes()] == ["w0", "w1", "w2", "w3"]
    assert [c.get_gpu("w%d" % g) for g in range(4)] == [0, 1, 2, 3]
    run = (tmp_path / "run.sh").read_text()
    assert run.startswith("#!/bin/bash")
    assert ("torchrun --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29500 main.py "
            "--lr=0.01 --batch-size 8 --config-file ./dpwa.yaml") in run
    assert os.stat(tmp_path / "run.sh").st_mode & stat.S_IEXEC
    name, dev = node_for_rank(str(cfg), rank=2)
    assert name == "w2" and dev.index == 2
    with pytest.raises(ValueError):
        node_for_rank(str(cfg), rank=4)


def test_gpu_key_places_the_node(tmp_path):
    """A node's gpu: key is checked against its parameters' device at bind time (on the GPU
    box, tests/test_gpu_configs.py checks the adapter moving a model onto that device)."""
    import torch
    from dpwa_amd.launch import write_config
    p = write_config(str(tmp_path / "g.yaml"), ["a", "b"], gpus=[1, 0])
    conn = DpwaConnection("a", p, group=LocalGroup())
    with pytest.raises(ValueError, match="gpu 1"):
        conn.update_send(torch.zeros(4, device="meta"), 1.0)
    conn.close()


def test_pull_modes_are_validated_before_binding(tmp_path):
    """set_pull accepts the transports DistGroup and the board offer (copy, kernel, relay,
    relay-avg, each with an optional block count) and refuses anything else; nothing touches
    the GPU before the connection is bound."""
    from dpwa_amd.launch import write_config
    cfg = write_config(str(tmp_path / "p.yaml"), ["a", "b"], interpolation="constant")
    conn = DpwaConnection("a", cfg, group=LocalGroup())
    for mode in ("copy", "kernel", "kernel:256", "relay", "relay:32", "relay-avg", "relay-avg:128"):
        conn.set_pull(mode)
        assert conn._pull == mode
    for bad in ("rccl", "relay_avg", "push:32", ""):
        with pytest.raises(ValueError, match="relay-avg"):
            conn.set_pull(bad)


def test_local_group_reaches_peers_by_address(tmp_path):
    """LocalGroup wires a peer entry to the learner that serves its address, as the reference's
    TxThread reaches whatever RxThread listens at (host, port) (conn.py:246-251): the self-peer
    (a node entry at the learner's own address), an alias of another learner, a name match, and a
    node nobody serves (refused); wiring follows learners joining and leaving."""
    from dpwa_amd import DpwaConnection, _lib
    from dpwa_amd.group import LocalGroup
    cfg = tmp_path / "alias.yaml"
    cfg.write_text("- nodes:\n"
                   "  - {name: a, host: localhost, port: 46100}\n"
                   "  - {name: b, host: 127.0.0.1, port: 46101}\n"
                   "  - {name: a-self, host: 127.0.0.1, port: 46100}\n"
                   "  - {name: ghost, host: localhost, port: 46199}\n"
                   "- fetch_probability: 1\n- timeout_ms: 2500\n- interpolation: constant\n"
                   "- divergence_threshold: 0\n- constant: { value: 0.5 }\n- clock: 0\n- loss: 0\n")
    group = LocalGroup()
    a = DpwaConnection("a", str(cfg), seed=1, group=group)
    L, U = _lib.NODE_PEER_LOCAL, _lib.NODE_PEER_UNSET
    # a's peers: b (not there yet), a-self (a itself), ghost (nobody)
    assert [p.name for p in a.peers] == ["b", "a-self", "ghost"]
    assert a._peer_wiring == [(U, None), (L, "a"), (U, None)]
    b = DpwaConnection("b", str(cfg), seed=2, group=group)
    assert a._peer_wiring == [(L, "b"), (L, "a"), (U, None)]
    # b's peers: a, a-self (a's address: a), ghost
    assert b._peer_wiring == [(L, "a"), (L, "a"), (U, None)]
    a.close()
    assert b._peer_wiring == [(U, None), (U, None), (U, None)]
    b.close()
