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
