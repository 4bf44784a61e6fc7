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


def test_two_ranks_report_the_reference_loop_and_a_shared_device_xgmi_line():
    """The driver's N>1 line with the write-through learner set on (secondary publish form and the
    overlap leg, which run the reference's loop order beside the resident timed run): the line's
    last key is `reference_loop` with a write-through value, the overlap names its publish form,
    and with both ranks on one GPU the xGMI block says so and leaves `frac` null."""
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
    assert list(out)[-1] == "reference_loop"
    ref = out["reference_loop"]
    assert ref["publish"] == "write-through" and ref["value"] > 0 and "resident" in ref["headline"]
    assert out["secondary_publish"]["publish"] == "write-through"
    assert out["overlap"]["publish"] == "write-through" and out["overlap"]["ms_per_step"] > 0
    x = out["xgmi"]
    assert x["peak_gbs"] == 76.8 and x["ranks_share_device"] is True and x["frac"] is None


def test_injected_transport_failure_is_isolated():
    # the timed rounds run resident learners (the default publish form): their transport fails
    rc, lines, err = _bench({"DPWA_BENCH_INJECT": "lockstep/kernel:256+res@1:end"})
    assert rc == 1, err[-3000:]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["parity"]["lockstep/kernel:256+res"] is False
    assert all(v for k, v in out["parity"].items() if k not in ("workload", "lockstep/kernel:256+res"))
    assert out["value"] > 0 and not any(k.startswith("kernel") for k in out["pull_trials_gbs"])


def test_resident_parity_failure_falls_back_to_write_through():
    """If no resident transport passes the parity check (here an injected failure in the N=1 leg's
    `local+res`), the timed run uses the verified write-through form, says so in the line, and the
    run still exits 1 for the failed transport."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["DPWA_BENCH_INJECT"] = "local+res@0:end"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2",
                        "--no-cpu-baseline", "--no-sweep", "--compute-us", "0", "--no-secondary", "--no-cold"],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert p.returncode == 1, p.stderr[-3000:]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["parity"]["local+res"] is False and out["parity"]["local"] is True
    assert "publish_fallback" in out and out["config"]["publish"] == "write-through"
    assert out["value"] > 0 and out["parity_of_timed_transport"] == {"transport": "local", "ok": True}


def test_one_gpu_line_prices_the_mutual_pair_on_algorithmic_and_hbm_bytes():
    """N=1 resident: the two learners average with each other in one dispatch, so the roofline
    counts §8(d)'s 3*N*s per averaging for both (6*N*s, `bytes_per_launch`, `achieved`, `frac`)
    and, in `hbm`, the 4*N*s the shared reads leave to move; both rates come from one launch time."""
    n = 1_000_003
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--numel", str(n), "--steps", "5",
                        "--warmup", "2", "--no-cpu-baseline", "--no-sweep", "--compute-us", "0", "--no-secondary"],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(lines[0])
    r = out["roofline"]
    assert out["config"]["publish"] == "resident" and r["learners_per_launch"] == 2 and r["cold"]["mutual_pair"]
    assert r["bytes_per_launch"] == 6 * n * 4 and r["hbm"]["bytes_per_launch"] == 4 * n * 4
    assert abs(r["achieved"] / r["hbm"]["achieved"] - 1.5) < 1e-3
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3 and r["hbm"]["traffic_x"] is None
