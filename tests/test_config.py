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
    """The generated file follows the reference schema: the reference's own parser
    (re-stated in config.json's fixtures) yields the same dict as ours for the same text."""
    from dpwa_amd.launch import write_config
    p = write_config(str(tmp_path / "g.yaml"), ["a", "b"], interpolation="loss", divergence_threshold=0.5)
    c = DpwaConfiguration(p)
    assert set(c.config) == {"nodes", "fetch_probability", "timeout_ms", "interpolation", "divergence_threshold",
                             "constant", "clock", "loss"}
