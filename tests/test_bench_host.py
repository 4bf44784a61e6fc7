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
    assert bench.parity_transports(1) == ["self", "local", "local+res"]
    t = bench.parity_transports(8)
    assert "lockstep/relay-avg:32+vmm" in t and "async/copy+vmm" in t
    assert "lockstep/relay-avg:32+res+vmm" in t and "async/copy+res+vmm" in t
    # the provisional N>1 line is measured right after the first transport, which must be the plain
    # copy-engine pull (main() checks it alone, then the rest)
    assert t[0] == "lockstep/copy" and bench.parity_transports(8, "lockstep")[0] == "lockstep/copy"
    lockstep = ["copy", "kernel:256", "kernel:1024", "relay:32", "relay:128", "relay:512", "relay-avg:32",
                "relay-avg:128", "relay-avg:512"]
    trials = lockstep + ["async/%s%s" % (m, wt) for m in lockstep if not m.startswith("relay") for wt in ("", "+wt")]
    # resident learners (the default publish form): "+res" trial keys, vouched for by "+res" transports
    trials += [m + "+res" for m in lockstep] + ["async/%s+res" % m for m in lockstep if not m.startswith("relay")]
    assert {bench.parity_key(k) for k in trials} <= set(t)
    assert bench.parity_key("relay-avg:512+res") == "lockstep/relay-avg:32+res"
    assert bench.parity_key("async/kernel:1024+res") == "async/kernel:256+res"
    assert bench.trial_mode("relay-avg:128+res") == "relay-avg:128" and bench.trial_mode("async/copy+wt") == "copy"
    assert all(x.startswith("async/") for x in bench.parity_transports(4, "async"))
    assert all(x.startswith("lockstep/") for x in bench.parity_transports(4, "lockstep"))


def test_write_through_learners_are_vouched_for():
    """A resident run times the reference loop's write-through form on a second set of learners
    with the chosen pull: the parity transport checked for it exists for every possible choice."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    assert bench.write_through_key(1, "auto") == "local"
    lockstep = ["copy", "kernel:256", "kernel:1024", "relay:32", "relay:128", "relay-avg:512"]
    chosen = [m + "+res" for m in lockstep] + ["async/%s+res" % m for m in lockstep if not m.startswith("relay")]
    t = set(bench.parity_transports(8))
    for c in chosen:
        k = bench.write_through_key(8, c)
        assert k in t and "+res" not in k, (c, k)
    assert bench.write_through_key(8, "async/kernel:1024+res") == "async/kernel:256+wt"
    assert bench.write_through_key(8, "relay-avg:512+res") == "lockstep/relay-avg:32"


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


def _watchdog_child(held, rc, detail=None):
    """A process whose watchdog overruns a 0.05 s phase after hold(held, rc)."""
    import subprocess
    env = dict(os.environ)
    if detail:
        env["DPWA_BENCH_DETAIL"] = str(detail)
    code = ("import sys, time, json; sys.path.insert(0, %r); import bench\n"
            "wd = bench.Watchdog(bench.parse(['--gpus', '1']), 1, 0)\n"
            "wd.hold(%s, %s)\n"
            "wd.enter('dist round sweep 7000000000 bf16', 0.05)\n"
            "time.sleep(30)\n" % (ROOT, held, rc))
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, env=env)


def test_overrun_after_the_measurement_prints_the_finished_line(tmp_path):
    """An overrun in the sweeps (after the timed measurement) prints the line built so far with
    the error added and exits with the run's own status (0, or 1 for a failed parity check); the
    sweep rows measured so far are in the detail file the line names."""
    import json
    det = tmp_path / "detail.json"
    p = _watchdog_child("{'value': 5200.0, 'round_sweep': [{'numel': 11173962, 'value': 5100.0}]}", 0, det)
    assert p.returncode == 0, p.stderr
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 5200.0 and "round_sweep" not in d and d["detail"] == str(det)
    assert json.loads(det.read_text())["round_sweep"][0]["value"] == 5100.0
    assert "overran" in d["error"] and d["phase"].startswith("dist round sweep")
    p = _watchdog_child("None", 1)           # a rank other than 0 (no line), parity failed
    assert p.returncode == 1 and not p.stdout.strip()
    p = _watchdog_child("None", "None")      # before the measurement: the partial line, status 3
    assert p.returncode == 3
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["value"] is None and "overran" in d["error"]


def test_committed_pmc_traffic_is_found_for_the_line_kernels():
    """The bench line's `roofline.traffic` and `reference_loop.kernel_cold[*].traffic_x` come from
    committed PMC summaries (profiles/traffic_<round>_*.json, newest round first); each of the
    cold kernels of configs[1] has one, within 0.1 % of its algorithmic bytes -- the mutual pair
    (two resident learners reading each other's slot, XCD-grouped) at its distinct 4*N*s."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    n = bench.RESNET18_NUMEL
    for publish, learners, per in (("resident", 2, 3), ("resident", 1, 3), ("write-through", 2, 4),
                                   ("write-through", 1, 4), ("resident-pair", 2, 2)):
        tb, src = bench.pmc_traffic(None, publish, learners, n, "f32", "cold")
        assert tb and src.startswith("profiles/traffic_"), (publish, learners)
        assert abs(tb / (learners * per * n * 4) - 1) < 1e-3, (publish, learners, tb)
    assert bench.pmc_traffic(None, "resident", 2, n + 1, "f32", "cold") == (None, None)


def test_scaling_basis_has_one_schema_at_every_n():
    """`scaling_basis` (raw and weak rounds/s, one learner per GPU) carries the same keys at N=1, 2 and
    8, with and without the overlap leg, so the driver's per-N lines compare like with like."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    ov = {"gossip_rounds_per_s": 800.0, "ms_per_step": 1.2, "compute_only_ms_per_step": 1.19,
          "gossip_overhead_frac": 0.008}
    shapes = set()
    for world in (1, 2, 8):
        for overlap in (ov, None):
            sb = bench.scaling_basis(world, 1, "write-through", 20.0 * world, 0.001, 5000.0, overlap)
            shapes.add((tuple(sorted(sb)), tuple(sorted(sb["raw"])), tuple(sorted(sb["weak"]))))
            assert sb["learners"] == world and sb["raw"]["gossip_rounds_per_s"] == 20000.0 * world
            assert sb["raw"]["gossip_rounds_per_s_per_learner"] == 20000.0
            if overlap:
                assert sb["weak"]["gossip_rounds_per_s_per_learner"] == round(800.0 / world, 1)
            else:
                assert sb["weak"]["gossip_rounds_per_s"] is None
    assert len(shapes) == 1


def test_self_peer_config_is_the_reference_schema(tmp_path):
    """bench's configs[1] YAML: the learner and a second entry at its own host:port; parsed by the
    reference-schema reader, the learner's only peer is that entry, at the learner's own address."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    from dpwa_amd.dpwa import DpwaConfiguration
    cfg = tmp_path / "c.yaml"
    bench.write_config(str(cfg), ["w1"], "constant", self_peer=True, base_port=45123)
    nodes = DpwaConfiguration(str(cfg)).get_nodes()
    assert [n["name"] for n in nodes] == ["w1", "w1-self"]
    assert {(n["host"], n["port"]) for n in nodes} == {("127.0.0.1", 45123)}


def _worst_case_result(world):
    """A full result as large as the N>1 run can make it: every parity transport, every trial
    key, an xGMI block with the relay, long notes and sweeps, a CPU baseline with rows."""
    import bench
    note = "x" * 900
    parity = {t: True for t in bench.parity_transports(world)}
    parity.update({"extra/transport-%02d" % i: (i % 3 != 0) for i in range(40)})
    parity["workload"] = note
    sweep = [{"numel": 7_000_000_000, "dtype": "bf16", "value": 1.0, "note": note} for _ in range(12)]
    sb = bench.scaling_basis(world, 1, "write-through", 20.0 * world, 0.001, 5000.0,
                             {"gossip_rounds_per_s": 800.0, "ms_per_step": 1.2, "compute_only_ms_per_step": 1.19,
                              "gossip_overhead_frac": 0.008})
    return {**bench.base_line(bench.parse(["--gpus", str(world)]), world),
            "value": 1234.5, "ms_per_step": 0.5, "value_cold": {"value": 1000.0, "note": note},
            "scaling_basis": sb, "gossip_rounds_per_s": 1.0, "gossip_rounds_per_s_per_learner": 1.0,
            "averagings": 20, "round_sweep": sweep, "warmup_rounds": {"note": note},
            "roofline": {"bound": "hbm", "achieved": 6000.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.75,
                         "traffic": 1.0e8, "traffic_x": 1.0, "bytes_per_launch": 178_783_392, "kernel": note,
                         "avg_launch_us": 28.0, "in_loop_frac": 0.8, "mix_ceiling_frac": 0.77,
                         "size_sweep": sweep, "in_loop": {"note": note}, "mix_ceiling": {"note": note}},
            "config": {"workload": note, "numel": 11_173_962, "publish": "write-through", "peer": note,
                       "loop_order": note, "learners": world},
            "cpu_baseline": {"value": 2.4, "unit": "GB/s", "cores": 2, "kind": "port", "ms_per_round": 109.7,
                             "sample": note, "rows": sweep, "restatement_rows": sweep, "phases_note": note},
            "parity": parity, "parity_of_timed_transport": {"transport": "lockstep/copy", "ok": True},
            "pull_trials_gbs": {"t%d" % i: [1.0] * 10 for i in range(30)},
            "pull_choice": {"chosen": "relay-avg:128", "rule": note},
            "trial_errors": {"t%d" % i: note for i in range(30)},
            "xgmi": {"bytes_per_pull": 1, "avg_pull_us": 2.0, "achieved_gbs_per_pull": 50.0, "peak_gbs": 76.8,
                     "frac": 0.6, "ranks_share_device": False, "note": note,
                     "relay": {"frac": 0.5, "note": note}},
            "overlap": {"note": note}, "secondary_publish": {"note": note}, "adapter_loop": {"note": note},
            "co_resident_pair": {"note": note}, "publish_fallback": note}


def test_result_line_is_bounded_scalar_and_keeps_the_headline():
    """The line the driver parses (round 5's was cut at 21.7 KB): at most LINE_MAX bytes for the
    largest result either N can build, scalar blocks only, the headline figures kept."""
    import json
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 8):
        full = _worst_case_result(world)
        line = json.dumps(bench.compact_line(full, "gpurun_out/bench_detail_n%d.json" % world))
        assert len(line.encode()) <= bench.LINE_MAX, (world, len(line))
        d = json.loads(line)
        assert d["value"] == 1234.5 and d["value_cold"] == 1000.0 and d["detail"].endswith(".json")
        assert d["roofline"]["frac"] == 0.75 and d["roofline"]["traffic_x"] == 1.0
        assert d["cpu_baseline"]["value"] == 2.4 and d["cpu_baseline"]["cores"] == 2
        assert d["parity_of_timed_transport"]["ok"] is True
        assert d["scaling_basis"]["raw"]["gossip_rounds_per_s"] == 20000.0 * world
        for block in ("roofline", "config", "cpu_baseline", "xgmi"):
            if block in d:
                assert not any(isinstance(v, (dict, list)) for v in d[block].values()), block
        assert "round_sweep" not in d and "adapter_loop" not in d


def test_provisional_line_is_a_bounded_contract_line():
    """The N>1 provisional line (bench.provisional_line's shape): the contract keys, `provisional`
    and its verified transport kept in the compact line, and an error added when it is printed."""
    import json
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench

    class A:
        steps, warmup, dtype, numel, interpolation, fetch_probability = 20, 5, "f32", 11_173_962, "constant", 1.0

    out = bench.base_line(A, 8)
    parity = {t: True for t in bench.parity_transports(8)}
    out.update({"value": 900.0, "ms_per_step": 1.2, "gossip_rounds_per_s": 6666.7, "averagings": 160,
                "provisional": True,
                "roofline": {"bound": "hbm", "achieved": None, "peak": 8000.0, "unit": "GB/s", "frac": None,
                             "traffic": None, "bytes_per_launch": 4 * A.numel * 4, "avg_launch_us": None,
                             "kernel": "k"},
                "scaling_basis": {"n_gpus": 8, "raw": {"gossip_rounds_per_s": 6666.7, "value": 900.0}, "weak": {}},
                "config": {"workload": "w", "pull": "lockstep/copy", "numel": A.numel},
                "parity": parity, "parity_of_timed_transport": {"transport": "lockstep/copy", "ok": True},
                "error": "watchdog: phase 'parity lockstep/kernel:256' overran its budget (the line up to it)",
                "phase": "parity lockstep/kernel:256"})
    d = json.loads(json.dumps(bench.compact_line(out, "gpurun_out/bench_detail_n8.json")))
    assert len(json.dumps(d)) <= bench.LINE_MAX
    assert d["provisional"] is True and d["value"] == 900.0 and d["error"].startswith("watchdog")
    assert d["parity_of_timed_transport"] == {"transport": "lockstep/copy", "ok": True}
    assert d["config"]["pull"] == "lockstep/copy" and d["roofline"]["bytes_per_launch"] == 4 * A.numel * 4


def test_result_line_from_the_committed_round5_line():
    """Round 5's own 21.7 KB line (profiles/r05q_bench.json), compacted: within the bound."""
    import json
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    path = os.path.join(ROOT, "profiles", "r05q_bench.json")
    if not os.path.exists(path):
        return
    full = json.load(open(path))
    d = bench.compact_line(full, "x.json")
    assert len(json.dumps(d)) <= 4096, len(json.dumps(d))
    assert d["value"] == full["value"] and d["roofline"]["frac"] == full["roofline"]["frac"]
    assert d["cpu_baseline"]["value"] == full["cpu_baseline"]["value"]
    assert d["value_cold"] == full["value_cold"]["value"]


def test_vmm_threshold_matches_the_learner():
    """bench.VMM_MIN_BYTES (which N>1 sweep sizes use fd-shared slots, skipped when a +vmm parity
    transport failed) is learner.cpp's kVmmMinBytes."""
    import re
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    src = open(os.path.join(ROOT, "dpwa_amd", "csrc", "learner.cpp")).read()
    m = re.search(r"kVmmMinBytes = \(size_t\)(\d+) << (\d+);", src)
    assert m and bench.VMM_MIN_BYTES == int(m.group(1)) << int(m.group(2))
