"""bench.py's N>1 path as the driver starts it, on one GPU over gloo (RCCL refuses two ranks per
GPU): `python bench.py --gpus 2` with no launcher starts torch.distributed.run as a child and
must print exactly one result line, every parity transport true; an exception injected at the
end of one transport on one rank must turn into that transport's `false` with the line still
printed; the exit status is 1 only when the timed transport itself failed."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

ARGS = ["--gpus", "2", "--dist-backend", "gloo", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-sweep",
        "--compute-us", "0", "--no-secondary", "--trial-passes", "1", "--trial-ms", "5"]


LINE_MAX = 6144     # the driver keeps ~9 KB of stdout: the line stays well inside it
LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "config", "roofline", "scaling_basis", "parity", "parity_of_timed_transport",
             "detail")
ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "bytes_per_launch", "avg_launch_us", "kernel")


def _env(tmp, extra_env=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["DPWA_BENCH_DETAIL"] = str(tmp)
    env.update(extra_env or {})
    return env


def _line(lines):
    """The one result line: bounded, parseable, scalar-only, naming its detail file."""
    assert len(lines) == 1, lines
    assert len(lines[0].encode()) <= LINE_MAX, len(lines[0])
    out = json.loads(lines[0])
    for k in LINE_KEYS:
        assert k in out, k
    for block in ("roofline", "config", "cpu_baseline", "parity", "parity_of_timed_transport"):
        if isinstance(out.get(block), dict):
            assert all(not isinstance(v, (dict, list)) for v in out[block].values()), (block, out[block])
    return out


def _detail(out):
    with open(os.path.join(ROOT, out["detail"]) if not os.path.isabs(out["detail"]) else out["detail"]) as f:
        return json.load(f)


def _bench(tmp_path, extra_env=None, args=ARGS):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                       env=_env(tmp_path / "detail.json", extra_env),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    return p.returncode, lines, p.stderr


def test_self_launched_two_ranks_print_one_line(tmp_path):
    rc, lines, err = _bench(tmp_path)
    assert rc == 0, err[-3000:]
    out = _line(lines)
    assert out["n_gpus"] == 2 and out["value"] > 0
    parity = out["parity"]
    sys.path.insert(0, ROOT)
    import bench
    assert set(parity) == set(bench.parity_transports(2)) and all(parity.values()), parity
    assert out["parity_of_timed_transport"]["ok"]
    assert "provisional" not in out and "error" not in out     # the final line replaced the provisional one


def _scaling_schema(out):
    sb = out["scaling_basis"]
    return (sorted(sb), sorted(sb["raw"]), sorted(sb["weak"]), sb["learners_per_gpu"], sb["publish"])


def test_two_ranks_report_scaling_basis_and_a_shared_device_xgmi_line(tmp_path):
    """The driver's N>1 line with the overlap leg on: one learner per rank in the write-through
    form (the reference's loop order), `scaling_basis` with raw and weak rounds/s under the same
    keys as the N=1 line, the overlap names its publish form, and with both ranks on one GPU the
    xGMI block says so and leaves `frac` null."""
    args = [a for a in ARGS if a not in ("--no-secondary",)]
    i = args.index("--compute-us")
    args[i + 1] = "300"
    rc, lines, err = _bench(tmp_path, args=args)
    assert rc == 0, err[-3000:]
    out = _line(lines)
    det = _detail(out)
    assert out["config"]["publish"] == "write-through" and out["config"]["learners_per_gpu"] == 1
    sb = out["scaling_basis"]
    assert sb["learners_per_gpu"] == 1 and sb["publish"] == "write-through" and sb["n_gpus"] == 2
    assert sb["raw"]["gossip_rounds_per_s"] > 0 and sb["weak"]["gossip_rounds_per_s"] > 0
    assert out["config"]["scaling_weak_rounds_per_s"] == sb["weak"]["gossip_rounds_per_s"]
    assert det["secondary_publish"]["publish"] == "full"
    assert det["overlap"]["publish"] == "write-through" and det["overlap"]["ms_per_step"] > 0
    assert out["roofline"]["frac"] <= 1.0 and out["roofline"]["bytes_per_launch"] == 4 * 1 * 4 * 11_173_962
    x = out["xgmi"]
    assert x["peak_gbs"] == 76.8 and x["ranks_share_device"] is True and x["frac"] is None
    assert det["scaling_basis"]["definition"] and det["value"] == out["value"]
    # the N=1 line's scaling block has the same schema
    rc, lines, err = _bench(tmp_path, args=["--numel", "1000003", "--steps", "5", "--warmup", "2",
                                            "--no-cpu-baseline", "--no-sweep", "--compute-us", "300",
                                            "--no-secondary", "--no-value-cold"])
    assert rc == 0, err[-3000:]
    out1 = _line(lines)
    assert _scaling_schema(out1) == _scaling_schema(out)


def test_injected_transport_failure_is_isolated(tmp_path):
    # the timed rounds run write-through learners (the default publish form): their transport fails
    rc, lines, err = _bench(tmp_path, {"DPWA_BENCH_INJECT": "lockstep/kernel:256@1:end"})
    assert rc == 0, err[-3000:]          # the timed transport passed: the verified line stands
    assert "parity check FAILED for ['lockstep/kernel:256']" in err
    out = _line(lines)
    assert out["parity"]["lockstep/kernel:256"] is False and out["parity_failed"] == ["lockstep/kernel:256"]
    assert out["parity_of_timed_transport"]["ok"]
    assert all(v for k, v in out["parity"].items() if k != "lockstep/kernel:256")
    assert out["value"] > 0 and not any(k.startswith("kernel") for k in _detail(out)["pull_trials_gbs"])


def test_hang_in_a_late_parity_transport_keeps_the_measured_line(tmp_path):
    """At N>1 the fd-shared (+vmm) transports are checked after the line is held: a hang in one
    (here rank 1 raises at its start, so rank 0 blocks in the transport's first collective) ends
    the job through the watchdog with the measured line, that transport false, exit status 0.
    Whichever rank's watchdog fires first, rank 0 keeps the line: by its own watchdog, or by the
    post-measurement guard when rank 1's exit breaks the collective it is blocked in."""
    t = "lockstep/relay-avg:32+vmm"
    rc, lines, err = _bench(tmp_path, {"DPWA_BENCH_INJECT": "%s@1:start" % t}, args=ARGS + ["--phase-scale", "0.1"])
    assert rc == 0, err[-3000:]
    out = _line(lines)
    assert out["value"] > 0 and out["parity_of_timed_transport"]["ok"]
    assert out["parity"][t] is False and t in out["parity_failed"]
    assert ("watchdog" in out["error"] or "after the measurement" in out["error"]), out["error"]
    assert out["phase"] == "parity %s" % t
    assert all(v for k, v in out["parity"].items() if "+vmm" not in k)


def test_hang_before_the_final_measurement_leaves_the_provisional_line(tmp_path):
    """At N>1 lockstep/copy is checked first and the line's rounds are timed on it at once (the
    provisional line, held): a hang in a later transport (rank 1 raises at the start of
    lockstep/kernel:256, rank 0 blocks in its first collective) ends the job with that line --
    marked provisional, measured on the verified copy transport -- and that transport false."""
    t = "lockstep/kernel:256"
    rc, lines, err = _bench(tmp_path, {"DPWA_BENCH_INJECT": "%s@1:start" % t}, args=ARGS + ["--phase-scale", "0.1"])
    assert rc == 0, err[-3000:]
    out = _line(lines)
    assert out["provisional"] is True and out["value"] > 0 and out["ms_per_step"] > 0, out
    assert out["parity_of_timed_transport"] == {"transport": "lockstep/copy", "ok": True}
    assert out["parity"]["lockstep/copy"] is True and out["parity"][t] is False
    assert out["phase"] == "parity %s" % t, out["phase"]


def test_rank_lost_after_the_measurement_keeps_the_measured_line(tmp_path):
    """A rank that dies after the line is held (here rank 1 exits at a late parity transport):
    torch.distributed.run stops rank 0 with SIGTERM or rank 0's collective fails first; either
    way rank 0 leaves the measured line on stdout (its last words, or the exception path), with
    the phase it reached; the job's status is the launcher's.  The SIGTERM can arrive while rank 0
    is still registering the transport's phase: the line written is then the previous phase's,
    complete (the library keeps two buffers)."""
    t = "lockstep/relay-avg:32+vmm"
    rc, lines, err = _bench(tmp_path, {"DPWA_BENCH_INJECT": "%s@1:die" % t}, args=ARGS + ["--phase-scale", "0.2"])
    out = _line(lines)
    assert out["value"] > 0 and out["parity_of_timed_transport"]["ok"], err[-3000:]
    assert "ended by a signal" in out["error"] or "after the measurement" in out["error"], out["error"]
    assert out["phase"] in ("parity %s" % t, "report"), out["phase"]
    if out["phase"] != "report":
        assert out["parity"][t] is False


def test_resident_parity_failure_falls_back_to_write_through(tmp_path):
    """If no resident transport passes the parity check (here injected failures in every lock-step
    `+res` transport of a --publish resident run), the timed run uses the verified write-through
    form, says so in the line, and reports the failed transports (exit status 0: the timed one
    passed)."""
    res = ["lockstep/copy+res", "lockstep/kernel:256+res", "lockstep/relay:32+res", "lockstep/relay-avg:32+res",
           "lockstep/relay-avg:32+res+vmm"]
    rc, lines, err = _bench(tmp_path, {"DPWA_BENCH_INJECT": ",".join("%s@1:end" % t for t in res)},
                            args=ARGS + ["--publish", "resident", "--gossip", "lockstep", "--pull", "copy", "--no-cold"])
    assert rc == 0, err[-3000:]
    assert "parity check FAILED" in err
    out = _line(lines)
    assert all(out["parity"][t] is False for t in res) and out["parity"]["lockstep/copy"] is True
    assert "publish_fallback" in out and out["config"]["publish"] == "write-through"
    assert out["value"] > 0 and out["parity_of_timed_transport"] == {"transport": "lockstep/copy", "ok": True}


def _one_gpu(tmp_path, n, *extra):
    rc, lines, err = _bench(tmp_path, args=["--numel", str(n), "--steps", "20", "--warmup", "5", "--no-cpu-baseline",
                                            "--no-sweep", "--compute-us", "0"] + list(extra))
    assert rc == 0, err[-3000:]
    out = _line(lines)
    return out, _detail(out)


def test_one_gpu_line_is_configs1_self_peer_within_the_roofline(tmp_path):
    """The N=1 line is configs[1] as BASELINE/SURVEY §8(d) C2 state it: one learner, its peer its own
    snapshot, the write-through form.  Its metric bytes over the step time and the roofline's
    fraction obey the HBM peak: value (3*N*s per averaging / wall time) <= 8 TB/s, roofline.frac
    (4*N*s moved / cold launch time / 8 TB/s) <= 1; value_cold rotates > 1.2 GB of learner sets;
    the co-resident pair's metric-unit rate sits in its own block with its HBM frac."""
    n = 11_173_962
    out, det = _one_gpu(tmp_path, n)
    assert out["config"]["publish"] == "write-through" and out["config"]["learners"] == 1
    assert out["parity_of_timed_transport"] == {"transport": "self", "ok": True}
    assert 3 * n * 4 / (out["ms_per_step"] * 1e-3) / 1e9 <= 8000.0
    assert out["value"] <= 8000.0
    r = out["roofline"]
    assert r["bytes_per_launch"] == 4 * n * 4 and r["metric_bytes_per_averaging"] == 3 * n * 4
    assert 0 < r["frac"] <= 1.0 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert abs(r["achieved"] / (r["bytes_per_launch"] / (r["avg_launch_us"] * 1e-6) / 1e9) - 1) < 1e-3
    # the same access mix alone, interleaved launch by launch on the same buffers: the product
    # kernel (factor, lerp, tail) runs at its mix's rate (round 5: 0.98-1.01 in tools/product_tune)
    mix = det["roofline"]["mix_ceiling"]
    assert mix["interleaved"] and mix["mix"] == "2R:2W" and mix["bytes_per_launch"] == 4 * (n * 4 // 16 * 16)
    assert 0 < mix["frac"] <= 1.0 and r["kernel_over_mix_ceiling"] >= 0.93, r
    vc = det["value_cold"]
    assert vc["bytes_between_reuses"] > 1.2e9 and 0 < vc["value"] <= 8000.0
    assert out["config"]["value_cold"] == vc["value"] == out["value_cold"]
    pair = det["co_resident_pair"]
    assert pair["learners"] == 2 and 0 < pair["hbm"]["frac"] <= 1.0
    # the drop-in adapter itself: its reuse guard (two small launches per update_send) stays a small
    # part of the round (round 5 measured 30.3 against 26.5 us; a single-workgroup compare took 45.9)
    ad = det["adapter_loop"]
    assert ad["default"]["reuse_guard"] and not ad["no_guard"]["reuse_guard"]
    assert ad["default"]["ms_per_step"] <= 1.35 * ad["no_guard"]["ms_per_step"], ad
    # the resident adapter's window guard (a save at update_send, a compare at update_wait) likewise
    assert ad["resident"]["resident"] and ad["resident"]["reuse_guard"] and ad["resident"]["guard_hits"] == 0
    assert ad["resident"]["ms_per_step"] <= 1.35 * ad["resident_no_guard"]["ms_per_step"], ad


@pytest.mark.timeout(900)
def test_driver_command_prints_one_bounded_line(tmp_path):
    """The driver's exact N=1 command (`bench.py --gpus 1 --steps 20 --warmup 5`: CPU baseline,
    restatement rows, value_cold, side loops and both sweeps all on) prints one line of at most
    LINE_MAX bytes that json.loads, with the headline scalars; the sweeps and rows are in the
    detail file the line names.  (Round 5's 21.7 KB line was cut by the driver and left unparsed.)
    Progress goes to gpurun_out/ so a long run is visibly alive."""
    log_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(log_dir, exist_ok=True)
    with open(os.path.join(log_dir, "driver_command.err"), "w") as err:
        p = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--steps", "20", "--warmup", "5"], cwd=ROOT,
                           env=_env(tmp_path / "detail.json"), stdout=subprocess.PIPE, stderr=err, text=True,
                           timeout=880)
    assert p.returncode == 0
    out = _line([ln for ln in p.stdout.splitlines() if ln.strip()])
    for k in ROOFLINE_KEYS + ("in_loop_frac", "mix_ceiling_frac", "traffic_x"):
        assert k in out["roofline"], k
    assert out["roofline"]["bound"] == "hbm" and 0 < out["roofline"]["frac"] <= 1.0
    cpu = out["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] in ("port", "reference") and cpu["ms_per_round"] > 0
    assert 0 < out["value_cold"] <= 8000.0 and out["value"] > 0 and out["ms_per_step"] > 0
    assert set(out["scaling_basis"]) >= {"raw", "weak"} and out["parity_of_timed_transport"]["ok"]
    assert all(out["parity"].values()) and "error" not in out and "provisional" not in out
    det = _detail(out)
    assert det["value"] == out["value"] and det["cpu_baseline"]["restatement_rows"]
    assert det["roofline"]["size_sweep"] and det["round_sweep"]
