"""Host logic of bench.py that needs no GPU: which parity transport vouches for each transport
trial (at N>1 the parity leg runs before the trials and only verified transports are timed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_trial_maps_to_a_parity_transport():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    parity_transports = {"lockstep/copy", "lockstep/kernel:256", "lockstep/relay:32", "lockstep/relay-avg:32",
                         "async/copy",
                         "async/kernel:256", "async/copy+wt", "async/kernel:256+wt"}
    lockstep = ["copy", "kernel:256", "kernel:1024", "relay:32", "relay:128", "relay:512", "relay-avg:32",
                "relay-avg:128", "relay-avg:512"]
    trials = lockstep + ["async/%s%s" % (m, wt) for m in lockstep if not m.startswith("relay") for wt in ("", "+wt")]
    keys = {t: bench.parity_key(t) for t in trials}
    assert set(keys.values()) == parity_transports
    assert keys["kernel:1024"] == "lockstep/kernel:256"
    assert keys["relay:512"] == "lockstep/relay:32"
    assert keys["relay-avg:128"] == "lockstep/relay-avg:32"
    assert keys["async/kernel:1024+wt"] == "async/kernel:256+wt"
    assert keys["async/copy"] == "async/copy"


def test_parity_transports_cover_every_trial_and_the_fd_shared_path():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    assert bench.parity_transports(1) == ["local"]
    t = bench.parity_transports(8)
    assert "lockstep/relay-avg:32+vmm" in t and "async/copy+vmm" in t
    lockstep = ["copy", "kernel:256", "kernel:1024", "relay:32", "relay:128", "relay:512", "relay-avg:32",
                "relay-avg:128", "relay-avg:512"]
    trials = lockstep + ["async/%s%s" % (m, wt) for m in lockstep if not m.startswith("relay") for wt in ("", "+wt")]
    assert {bench.parity_key(k) for k in trials} <= set(t)
    assert all(x.startswith("async/") for x in bench.parity_transports(4, "async"))
    assert all(x.startswith("lockstep/") for x in bench.parity_transports(4, "lockstep"))


def test_injection_hook_parsing(monkeypatch):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("DPWA_BENCH_INJECT", "lockstep/relay:32@1:start,async/copy@0")
    assert bench.injected("lockstep/relay:32", 1, "start")
    assert not bench.injected("lockstep/relay:32", 1, "end")
    assert not bench.injected("lockstep/relay:32", 0, "start")
    assert bench.injected("async/copy", 0, "end")          # ":end" is the default
    monkeypatch.delenv("DPWA_BENCH_INJECT")
    assert not bench.injected("async/copy", 0, "end")


def test_partial_line_keeps_the_contract_keys():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    out = bench.base_line(bench.parse(["--gpus", "8", "--steps", "20", "--warmup", "5"]), 8)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data"):
        assert k in out
    assert out["n_gpus"] == 8 and out["steps"] == 20 and out["value"] is None
