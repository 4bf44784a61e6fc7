"""bench.py's N>1 path as the driver starts it, on one GPU over gloo (RCCL refuses two ranks per
GPU): `python bench.py --gpus 2` with no launcher starts torch.distributed.run as a child and
must print exactly one result line, every parity transport true; an exception injected at the
end of one transport on one rank must turn into that transport's `false` with the line still
printed and exit status 1."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

ARGS = ["--gpus", "2", "--dist-backend", "gloo", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-sweep",
        "--compute-us", "0", "--no-secondary", "--trial-passes", "1", "--trial-ms", "5"]


def _bench(extra_env=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS, cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    return p.returncode, lines, p.stderr


def test_self_launched_two_ranks_print_one_line():
    rc, lines, err = _bench()
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    parity = {k: v for k, v in out["parity"].items() if k != "workload"}
    sys.path.insert(0, ROOT)
    import bench
    assert set(parity) == set(bench.parity_transports(2)) and all(parity.values()), parity
    assert out["parity_of_timed_transport"]["ok"]


def _scaling_schema(out):
    sb = out["scaling_basis"]
    return (sorted(sb), sorted(sb["raw"]), sorted(sb["weak"]), sb["learners_per_gpu"], sb["publish"])


def test_two_ranks_report_scaling_basis_and_a_shared_device_xgmi_line():
    """The driver's N>1 line with the overlap leg on: one learner per rank in the write-through
    form (the reference's loop order), `scaling_basis` with raw and weak rounds/s under the same
    keys as the N=1 line, the overlap names its publish form, and with both ranks on one GPU the
    xGMI block says so and leaves `frac` null."""
    args = [a for a in ARGS if a not in ("--no-secondary",)]
    i = args.index("--compute-us")
    args[i + 1] = "300"
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["config"]["publish"] == "write-through" and out["config"]["learners_per_gpu"] == 1
    sb = out["scaling_basis"]
    assert sb["learners_per_gpu"] == 1 and sb["publish"] == "write-through" and sb["n_gpus"] == 2
    assert sb["raw"]["gossip_rounds_per_s"] > 0 and sb["weak"]["gossip_rounds_per_s"] > 0
    assert out["config"]["scaling_weak_rounds_per_s"] == sb["weak"]["gossip_rounds_per_s"]
    assert out["secondary_publish"]["publish"] == "full"
    assert out["overlap"]["publish"] == "write-through" and out["overlap"]["ms_per_step"] > 0
    assert out["roofline"]["frac"] <= 1.0 and out["roofline"]["bytes_per_launch"] == 4 * 1 * 4 * 11_173_962
    x = out["xgmi"]
    assert x["peak_gbs"] == 76.8 and x["ranks_share_device"] is True and x["frac"] is None
    # the N=1 line's scaling block has the same schema
    p1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--numel", "1000003", "--steps", "5",
                         "--warmup", "2", "--no-cpu-baseline", "--no-sweep", "--compute-us", "300", "--no-secondary",
                         "--no-value-cold"], cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                        text=True, timeout=280)
    assert p1.returncode == 0, p1.stderr[-3000:]
    out1 = json.loads([ln for ln in p1.stdout.splitlines() if ln.strip()][0])
    assert _scaling_schema(out1) == _scaling_schema(out)


def test_injected_transport_failure_is_isolated():
    # the timed rounds run write-through learners (the default publish form): their transport fails
    rc, lines, err = _bench({"DPWA_BENCH_INJECT": "lockstep/kernel:256@1:end"})
    assert rc == 1, err[-3000:]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["parity"]["lockstep/kernel:256"] is False
    assert all(v for k, v in out["parity"].items() if k not in ("workload", "lockstep/kernel:256"))
    assert out["value"] > 0 and not any(k.startswith("kernel") for k in out["pull_trials_gbs"])


def test_resident_parity_failure_falls_back_to_write_through():
    """If no resident transport passes the parity check (here injected failures in every lock-step
    `+res` transport of a --publish resident run), the timed run uses the verified write-through
    form, says so in the line, and the run still exits 1 for the failed transports."""
    res = ["lockstep/copy+res", "lockstep/kernel:256+res", "lockstep/relay:32+res", "lockstep/relay-avg:32+res",
           "lockstep/relay-avg:32+res+vmm"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["DPWA_BENCH_INJECT"] = ",".join("%s@1:end" % t for t in res)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS +
                       ["--publish", "resident", "--gossip", "lockstep", "--pull", "copy", "--no-cold"],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert p.returncode == 1, p.stderr[-3000:]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert all(out["parity"][t] is False for t in res) and out["parity"]["lockstep/copy"] is True
    assert "publish_fallback" in out and out["config"]["publish"] == "write-through"
    assert out["value"] > 0 and out["parity_of_timed_transport"] == {"transport": "lockstep/copy", "ok": True}


def _one_gpu(n, *extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--numel", str(n), "--steps", "20",
                        "--warmup", "5", "--no-cpu-baseline", "--no-sweep", "--compute-us", "0"] + list(extra),
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, lines
    return json.loads(lines[0])


def test_one_gpu_line_is_configs1_self_peer_within_the_roofline():
    """The N=1 line is configs[1] as BASELINE/SURVEY §8(d) C2 state it: one learner, its peer its own
    snapshot, the write-through form.  Its metric bytes over the step time and the roofline's
    fraction obey the HBM peak: value (3*N*s per averaging / wall time) <= 8 TB/s, roofline.frac
    (4*N*s moved / cold launch time / 8 TB/s) <= 1; value_cold rotates > 1.2 GB of learner sets;
    the co-resident pair's metric-unit rate sits in its own block with its HBM frac."""
    n = 11_173_962
    out = _one_gpu(n)
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
    mix = r["mix_ceiling"]
    assert mix["interleaved"] and mix["mix"] == "2R:2W" and mix["bytes_per_launch"] == 4 * (n * 4 // 16 * 16)
    assert 0 < mix["frac"] <= 1.0 and r["kernel_over_mix_ceiling"] >= 0.93, r
    vc = out["value_cold"]
    assert vc["bytes_between_reuses"] > 1.2e9 and 0 < vc["value"] <= 8000.0
    assert out["config"]["value_cold"] == vc["value"]
    pair = out["co_resident_pair"]
    assert pair["learners"] == 2 and 0 < pair["hbm"]["frac"] <= 1.0
    # the drop-in adapter itself: its reuse guard (two small launches per update_send) stays a small
    # part of the round (round 5 measured 30.3 against 26.5 us; a single-workgroup compare took 45.9)
    ad = out["adapter_loop"]
    assert ad["default"]["reuse_guard"] and not ad["no_guard"]["reuse_guard"]
    assert ad["default"]["ms_per_step"] <= 1.35 * ad["no_guard"]["ms_per_step"], ad
    # the resident adapter's window guard (a save at update_send, a compare at update_wait) likewise
    assert ad["resident"]["resident"] and ad["resident"]["reuse_guard"] and ad["resident"]["guard_hits"] == 0
    assert ad["resident"]["ms_per_step"] <= 1.35 * ad["resident_no_guard"]["ms_per_step"], ad
