#!/usr/bin/env python3
"""bench.py -- gossip-round throughput of the MI355X pairwise-averaging hot path.

A *step* is one gossip round of every learner in the job through the drop-in API:
``update_send`` (device clock += 1, snapshot publish, Bernoulli gate, peer choice, pull) then
``update_wait_average`` (device factor/clock, fused lerp that also writes the next snapshot).

Workload (BASELINE.json configs[1]): a synthetic 11,173,962-element fp32 parameter vector
(ResNet-18 size) per learner, N(0,1) data, constant interpolation 0.5, fetch_probability 1,
the adapter's default write-through form, one learner per GPU at every N.
  * ``--gpus 1``: one learner whose peer is its own snapshot -- configs[1]'s self-peer: its YAML
    has a second node entry at the learner's own host:port, which the reference's TxThread dials
    like any peer (conn.py:246-251), so it averages with what it published at update_send, read
    in place from HBM.  Beside it: ``value_cold`` (the same loop over learner sets rotated beyond
    the Infinity Cache) and ``co_resident_pair`` (two resident learners averaging with each other
    in one dispatch, round 4's line).
  * ``--gpus N``: one learner per GPU, one process per GPU.  Under an external launcher
    (``torch.distributed.run``, WORLD_SIZE set) every process is a rank; without one, this
    script starts ``torch.distributed.run`` itself as a child process (before anything touches
    a GPU), relays its output and exits with its code.  Peers' snapshot slots are mapped into
    each process (hipIpc handles; fds of hipMemCreate chunks from 1.5 GiB up) and pulled over
    xGMI on each learner's side stream.  Interleaved, wall-time-bounded trials of lock-step
    rounds (RCCL barrier; copy / kernel / relay pulls) and free-running rounds (gossip board)
    pick the transport of the timed run by the median rate.  Per-GPU work is fixed ->
    "scaling": "weak".  Every rank logs its phases to stderr (``[bench rN +s]``).

``value`` = algorithmic averaged bytes (3 * numel * sizeof(dtype) per completed averaging,
SURVEY.md §8d) summed over all learners / the max-over-ranks wall time of the K timed steps,
from a pass with no instrumentation.  ``roofline`` prices the averaging kernel alone, cold, per
launch (dispatch begin/end events) on the bytes it moves (4*N*s write-through, PMC-confirmed in
``traffic``); ``roofline.in_loop`` times the same kernel inside the loop in a separate sampled
pass.  ``scaling_basis`` carries the raw and weak (fixed training step) rounds/s with the same
keys at every N.  ``parity`` (before the timed rounds; at N>1 before the trials, so only
verified transports are timed) checks every transport bit for bit against the oracle, each
transport isolated (an error becomes ``false``, not a teardown), with a watchdog that prints a
partial line and exits non-zero if a phase overruns.  ``cpu_baseline`` times the reference's own
CPU round restated (oracle/ref_round.py: two learner processes on localhost TCP, pickle framing,
numpy fp32 lerp -- the path this one replaces) on the box's host cores before the GPU is
touched, and beside it the averaging arithmetic on the host (C oracle, numpy single thread,
torch-CPU on every thread) at every north_star size.
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

XGMI_LINK_GBS = 153.6          # MI355X xGMI per link (spec, both directions together)
XGMI_LINK_DIR_GBS = XGMI_LINK_GBS / 2   # one direction of one link: what a pull of a peer's snapshot uses
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_MEASURED_GBS = 6290.0      # the guide's measured HBM ceiling (float4 copy, MI355X_MICROARCH.md)
RESNET18_NUMEL = 11_173_962    # examples/pytorch-cifar/models/resnet.py ResNet18
REF_SAMPLE_MAX = 32_000_000    # cap on the reference-round CPU sample (elements)
NUMPY_SAMPLE_MAX = 1_000_000_000   # numpy single-thread rows above this run on a bounded chunk
# BASELINE.json north_star sizes, each in its config's dtype (configs[1..4])
SWEEP = ((RESNET18_NUMEL, "f32"), (100_000_000, "f32"), (1_000_000_000, "bf16"), (7_000_000_000, "bf16"))
METRIC = "pairwise-average GB/s (% HBM peak) + gossip rounds/s"
# The cold streaming ceiling of the write-through kernel's access mix (2 reads : 2 writes) at
# 11.17M fp32, per launch, measured by tools/stream_tune.hip (profiles/r02_stream_tune_11m.log).
MIX_CEILING_11M = {"mix": "2R:2W", "frac": 0.759, "source": "profiles/r02_stream_tune_11m.log ('dual 64x1')"}


_T0 = time.perf_counter()
_RESULT_FD = 1       # where the one result line goes (main() moves everything else off stdout)
_WATCHDOG = None     # main()'s, for the exception guard under __main__


def emit(line):
    """Writes the result line to the real stdout (a dup of fd 1 taken at start-up: libraries'
    banners -- gloo's "[Gloo] Rank k is connected", RCCL's -- were moved to stderr)."""
    data = (line + "\n").encode()
    while data:
        data = data[os.write(_RESULT_FD, data):]


def progress(msg):
    """One stderr line per phase and rank (stdout keeps the single JSON line)."""
    sys.stderr.write("[bench r%s +%.1fs] %s\n" % (os.environ.get("RANK", "0"), time.perf_counter() - _T0, msg))
    sys.stderr.flush()      # one write per line: ranks share the stream


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warmup-s", type=float, default=0.25,
                    help="after the W warmup steps, more untimed rounds until about this many seconds of rounds "
                         "have run (the same count on every rank), so the timed steps see steady-state clocks")
    ap.add_argument("--numel", type=int, default=RESNET18_NUMEL)
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32")
    ap.add_argument("--interpolation", choices=["constant", "clock", "loss"], default="constant")
    ap.add_argument("--fetch-probability", type=float, default=1.0)
    ap.add_argument("--divergence-threshold", type=float, default=0.0)
    ap.add_argument("--loss-schedule", choices=["constant", "decay"], default="constant",
                    help="reported loss: 1.0, or SURVEY §8d C4's 2exp(-t/200)+0.05U (crosses a threshold)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-rows", action="store_true",
                    help="skip the host averaging-arithmetic rows at every north_star size")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold-cache kernel measurement")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the sweeps over the north_star sizes (cold kernel, and whole rounds at N=1)")
    ap.add_argument("--publish", choices=["resident", "write-through", "full"], default="write-through",
                    help="how a round publishes and averages in the timed loop: write-through (the adapter's "
                         "default and the form the reference's loop order update_send -> step -> update_wait "
                         "needs: the averaging kernel also writes the next snapshot, 4*N*s, the publish moves "
                         "the header only), full (a 2*N*s snapshot copy every round, then the 3*N*s average) or, "
                         "at N>1, resident (the parameters live in the learner's two snapshot slots, 3*N*s; "
                         "needs update_send -> update_wait -> step)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the run of the other publish form and, at N=1, the co-resident pair")
    ap.add_argument("--no-value-cold", action="store_true",
                    help="skip value_cold (the timed loop over rotating learner sets, no Infinity-Cache reuse)")
    ap.add_argument("--no-write-through", action="store_true", help="same as --publish full --no-secondary")
    ap.add_argument("--no-batch", action="store_true",
                    help="N=1: one averaging dispatch per learner instead of one batched dispatch per round")
    ap.add_argument("--sample-every", type=int, default=4,
                    help="in-loop kernel timing pass: time the averaging dispatch every k-th step")
    ap.add_argument("--timing", choices=["dispatch", "bracket", "both"], default="dispatch",
                    help="averaging-kernel timing in the sampled pass: its own dispatch events "
                         "(hipExtLaunchKernelGGL), an event pair recorded around the launch, or both")
    ap.add_argument("--streams", default="one", choices=["one", "per-learner"],
                    help="stream per co-resident learner (their kernels may overlap; no batching) or one stream")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (gloo only to rehearse on one GPU)")
    ap.add_argument("--pull", default="auto",
                    help="N>1 fetch transport: copy (hipMemcpyAsync), kernel[:blocks], relay[:blocks] "
                         "(two-phase multi-link), or auto (median of interleaved trials)")
    ap.add_argument("--gossip", default="auto", choices=["auto", "lockstep", "async"],
                    help="N>1: lock-step rounds (DistGroup), free-running rounds (AsyncDistGroup, gossip "
                         "board), or trials of both keeping the faster")
    ap.add_argument("--trial-ms", type=float, default=50.0,
                    help="N>1: minimum wall time of one transport trial (and at least 30 rounds)")
    ap.add_argument("--trial-passes", type=int, default=3, help="N>1: interleaved passes over the candidates")
    ap.add_argument("--dist-sweep-max-numel", type=int, default=None,
                    help="N>1: leave sizes above this out of the round sweep (rehearsals with ranks sharing a GPU)")
    ap.add_argument("--compute-us", type=float, default=1000.0,
                    help="per-learner synthetic training step (bf16 GEMM loop) for the 'overlap' field; 0 = skip")
    ap.add_argument("--no-provisional", action="store_true",
                    help="N>1: no provisional lock-step copy measurement before the other transports are checked")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the parity leg (a short gossip through every transport, checked against the oracle)")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic summary (tools/pmc_traffic.py over rocprofv3 FETCH_SIZE/WRITE_SIZE passes of "
                         "tools/cold_sweep.py) to report; default profiles/traffic_r03_<publish form>.json")
    ap.add_argument("--phase-scale", type=float, default=1.0,
                    help="multiplies every watchdog phase budget (slow rehearsals)")
    ap.add_argument("--launch-timeout", type=float, default=3000.0,
                    help="self-launch (N>1 without torchrun): seconds before the child job is stopped")
    args = ap.parse_args(argv)
    if args.no_write_through:
        args.publish, args.no_secondary = "full", True
    return args


def base_line(args, world):
    """The keys every output line carries, the partial one included."""
    return {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic N(0,1) flat parameter vectors (no dataset needed)"}


# ---------------------------------------------------------------- the result line
# The driver keeps only the tail of stdout (about 9 KB): round 5's 21.7 KB line was cut and went
# unparsed.  The line therefore carries scalars only and stays under LINE_MAX bytes; everything
# else (sweeps, restatement rows, side loops, prose) goes to a detail file the line names.
LINE_MAX = 6144
_TOP = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "gossip_rounds_per_s", "gossip_rounds_per_s_per_learner", "averagings",
        "publish_fallback", "error", "phase", "provisional")
_ROOFLINE = ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_x", "bytes_per_launch",
             "metric_bytes_per_averaging", "avg_launch_us", "kernel", "in_loop_frac", "in_loop_avg_launch_us",
             "mix_ceiling_frac", "kernel_over_mix_ceiling", "learners_per_launch")
_CPU = ("value", "unit", "cores", "kind", "ms_per_round", "numel")
_XGMI = ("bytes_per_pull", "avg_pull_us", "achieved_gbs_per_pull", "peak_gbs", "frac", "ranks_share_device")
_SCALAR = (int, float, bool, str, type(None))


_SIZE_TAG = {11_173_962: "11m", 100_000_000: "100m", 1_000_000_000: "1b", 7_000_000_000: "7b"}


def _pick(d, keys, maxlen=160):
    """The scalar entries of `d` named in `keys` (strings cut to maxlen)."""
    out = {}
    for k in keys:
        v = (d or {}).get(k, None) if isinstance(d, dict) else None
        if k not in (d or {}) or not isinstance(v, _SCALAR):
            continue
        out[k] = v[:maxlen] if isinstance(v, str) else v
    return out


def compact_line(full, detail=None):
    """The driver's line from the full result: the contract keys and the scalar headline figures
    (value, roofline, cpu_baseline, value_cold, scaling_basis raw/weak, parity verdicts), at most
    LINE_MAX bytes.  `detail` = where the full result was written (named in the line)."""
    out = _pick(full, _TOP, maxlen=240)
    cfg = full.get("config")
    if isinstance(cfg, dict):
        out["config"] = {k: (v[:200] if isinstance(v, str) else v) for k, v in cfg.items()
                         if isinstance(v, _SCALAR) and k not in ("loop_order", "peer")}
        # north_star's table (GB/s and rounds/s at 11M / 100M / 1B / 7B) as scalars of `config`,
        # which the driver keeps: whole rounds at each size on the line's transport
        for row in full.get("round_sweep") or []:
            if isinstance(row, dict) and isinstance(row.get("value"), (int, float)):
                tag = _SIZE_TAG.get(row.get("numel"), str(row.get("numel")))
                out["config"]["sweep_%s_gbs" % tag] = row["value"]
                if isinstance(row.get("gossip_rounds_per_s"), (int, float)):
                    out["config"]["sweep_%s_rounds_per_s" % tag] = row["gossip_rounds_per_s"]
    vc = full.get("value_cold")
    out["value_cold"] = vc.get("value") if isinstance(vc, dict) else vc if isinstance(vc, _SCALAR) else None
    rl = full.get("roofline")
    if isinstance(rl, dict):
        out["roofline"] = _pick(rl, _ROOFLINE)
    cpu = full.get("cpu_baseline")
    if isinstance(cpu, dict):
        c = _pick(cpu, _CPU)
        if isinstance(cpu.get("sample"), str):
            c["sample"] = cpu["sample"][:360]
        out["cpu_baseline"] = c
    elif "cpu_baseline" in full:
        out["cpu_baseline"] = None
    sb = full.get("scaling_basis")
    if isinstance(sb, dict):
        s = _pick(sb, ("n_gpus", "learners_per_gpu", "learners", "publish"))
        for part in ("raw", "weak"):
            if isinstance(sb.get(part), dict):
                s[part] = {k: v for k, v in sb[part].items() if isinstance(v, (int, float, bool, type(None)))}
        out["scaling_basis"] = s
    par = full.get("parity")
    if isinstance(par, dict):
        out["parity"] = {k: bool(v) for k, v in par.items() if k != "workload"}
    pt = full.get("parity_of_timed_transport")
    if isinstance(pt, dict):
        out["parity_of_timed_transport"] = _pick(pt, ("transport", "ok"))
    x = full.get("xgmi")
    if isinstance(x, dict):
        out["xgmi"] = _pick(x, _XGMI)
        if isinstance(x.get("relay"), dict):
            out["xgmi"]["relay_frac"] = x["relay"].get("frac")
    pc = full.get("pull_choice")
    if isinstance(pc, dict):
        out["pull"] = pc.get("chosen")
    if isinstance(full.get("parity_failed"), list):
        out["parity_failed"] = full["parity_failed"][:24]
    if isinstance(full.get("trial_errors"), dict):
        out["trial_errors"] = sorted(full["trial_errors"])
    if detail:
        out["detail"] = detail
    # a hard bound whatever the content: shed the longest optional parts first
    for drop in (("config", "workload"), ("cpu_baseline", "sample"), ("roofline", "kernel"), ("trial_errors",),
                 ("config",), ("xgmi",), ("scaling_basis",), ("data",)):
        if len(json.dumps(out)) <= LINE_MAX:
            break
        if len(drop) == 2 and isinstance(out.get(drop[0]), dict):
            out[drop[0]].pop(drop[1], None)
        else:
            out.pop(drop[0], None)
    if len(json.dumps(out)) > LINE_MAX and isinstance(out.get("parity"), dict):
        p = out["parity"]
        out["parity"] = {"all": all(p.values()), "failed": [k for k, v in p.items() if not v][:20]}
    return out


def detail_path(world):
    """Where the full result goes: $DPWA_BENCH_DETAIL, else gpurun_out/bench_detail_n<N>.json."""
    return os.environ.get("DPWA_BENCH_DETAIL") or os.path.join(ROOT, "gpurun_out", "bench_detail_n%d.json" % world)


def result_line(full, path):
    """Writes the full result to `path` (best effort) and returns the compact line naming it."""
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path + ".tmp", "w") as f:
            json.dump(full, f, indent=1, default=str)
        os.replace(path + ".tmp", path)
        rel = os.path.relpath(path, ROOT)
        where = rel if not rel.startswith("..") else path
    except OSError as e:
        progress("detail file not written: %s" % e)
        where = None
    return json.dumps(compact_line(full, where))


def emit_result(full, path):
    """Writes the full result to `path` (best effort) and prints the compact line."""
    emit(result_line(full, path))


def emit_final(full, path):
    """Prints the held line exactly once: registered as the last words and flushed through the
    library, so a signal arriving now either finds it written or writes it itself, never both."""
    line = result_line(full, path)
    from dpwa_amd import _lib
    try:
        _lib.last_words(_RESULT_FD, line + "\n")
        _lib.last_words_flush()
        return
    except Exception as e:   # noqa: BLE001 -- the line goes out directly then
        progress("last words unavailable (%s): printing directly" % e)
    emit(line)


def set_last_words(full, path):
    """The held line as a signal would leave it (include/dpwa_hip.h dpwa_last_words_set): if the
    process is stopped from outside (torch.distributed.run stops every rank when one dies; a time
    limit) or dies in the runtime (a GPU fault ends in abort()) after the measurement, the line
    up to that phase is still written to stdout.  `full` None clears it."""
    from dpwa_amd import _lib
    try:
        _lib.last_words(_RESULT_FD, result_line(full, path) + "\n" if full is not None else "")
    except Exception as e:   # noqa: BLE001 -- best effort: the normal paths print the line anyway
        progress("last words not registered: %s" % e)


# ---------------------------------------------------------------- robustness of the N>1 run
def self_launch(args, argv):
    """`--gpus N` (N > 1) without an external launcher: run torch.distributed.run as a CHILD
    process (this process never touches a GPU and never re-execs), relay its stdout, and exit
    with its code.  If the job ends without a result line, print one saying so."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)
    progress("self-launch: %s" % " ".join(cmd[1:]))

    def orphan_guard():
        # in the child, before exec: if this process dies (even SIGKILL), torchrun gets SIGTERM and
        # stops its ranks, so no rank outlives the job on the GPU (Linux prctl PR_SET_PDEATHSIG = 1)
        try:
            ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM, 0, 0, 0)
        except Exception:   # noqa: BLE001 -- best effort
            pass

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, start_new_session=True, preexec_fn=orphan_guard)

    def forward(signum, _frame):   # a stop request for this process stops the whole job
        try:
            os.killpg(p.pid, signum)
        except ProcessLookupError:
            pass

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)

    def stop():
        progress("self-launch: %.0f s limit reached, stopping the job" % args.launch_timeout)
        for sig, wait in ((signal.SIGTERM, 15), (signal.SIGKILL, 0)):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                return
            try:
                p.wait(wait)
                return
            except subprocess.TimeoutExpired:
                pass

    timer = threading.Timer(args.launch_timeout, stop)
    timer.daemon = True
    timer.start()
    got = False
    for line in p.stdout:   # the result line to stdout, anything else the ranks print to stderr
        if line.lstrip().startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
            got = True
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = p.wait()
    timer.cancel()
    if not got:
        out = base_line(args, args.gpus)
        out["error"] = "torch.distributed.run exited with %d without a result line" % rc
        emit(json.dumps(out))
        rc = rc or 1
    return rc


class Watchdog:
    """Per-rank deadline on the current phase.  When a phase overruns (a hung collective, a
    stalled pull, a rank that died inside a collective), rank 0 prints the partial result line
    (phase reached, parity so far, the phase's transport false), every rank dumps its threads,
    and the process exits with status 3 -- so the job ends within the bound with a line."""

    def __init__(self, args, world, rank):
        self.args, self.world, self.rank = args, world, rank
        self.phase, self.deadline = "start", None
        self.parity = {}
        self.transport = None
        self.held, self.held_rc = None, None   # hold(): the finished line and the run's exit status
        self.fired = self.disarmed = False
        self._lock = threading.Lock()
        t = threading.Thread(target=self._run, name="bench-watchdog", daemon=True)
        t.start()

    def enter(self, phase, seconds, transport=None):
        with self._lock:
            self.phase = phase
            self.transport = transport
            self.deadline = time.monotonic() + seconds * self.args.phase_scale
            held = self.held
        progress(phase)
        if held is not None:
            self._last_words(held, phase, transport)

    def hold(self, result, rc):
        """From here on an overrun prints `result` (rank 0's finished line; None on other ranks)
        with the phase and the error added, and exits with `rc`; hold(None, None) undoes it.
        While a line is held it is also registered as the process's last words (set_last_words),
        refreshed at every phase; hold(None, ...) clears them."""
        with self._lock:
            self.held, self.held_rc = result, rc
            phase, transport = self.phase, self.transport
        if self.rank == 0 and (result is not None or self._words):
            self._last_words(result, phase, transport)

    _words = False

    def _last_words(self, held, phase, transport):
        if self.rank != 0:
            return
        if held is None:
            set_last_words(None, None)
            self._words = False
            return
        out = dict(held)
        out["error"] = ("ended by a signal in phase '%s', %s" % (phase, "before the full measurement (the provisional line)"
                        if held.get("provisional") else "after the measurement (the line up to it)"))
        out["phase"] = phase
        if transport is not None and isinstance(out.get("parity"), dict):
            out["parity"] = dict(out["parity"], **{transport: False})
        set_last_words(out, detail_path(self.world))
        self._words = True

    def idle(self):
        with self._lock:
            self.deadline = None

    def disarm(self):
        """Stops the watchdog for good; False when it has already fired (it prints and exits)."""
        with self._lock:
            if self.fired:
                return False
            self.deadline, self.disarmed = None, True
            return True

    def _run(self):
        import faulthandler
        while True:
            time.sleep(1.0)
            with self._lock:
                late = not self.disarmed and self.deadline is not None and time.monotonic() > self.deadline
                self.fired = self.fired or late
                phase, transport = self.phase, self.transport
                held, held_rc = self.held, self.held_rc
            if not late:
                continue
            progress("WATCHDOG: phase '%s' overran its budget; exiting" % phase)
            if held_rc is not None:      # the measurement is complete: the line as it stands
                if held is not None:
                    out = dict(held)
                    out["error"] = "watchdog: phase '%s' overran its budget (the line up to it)" % phase
                    out["phase"] = phase
                    if transport is not None and isinstance(out.get("parity"), dict):   # a late parity check
                        out["parity"] = dict(out["parity"], **{transport: False})
                        out["parity_failed"] = sorted(k for k, v in out["parity"].items()
                                                      if k != "workload" and not v)
                    emit_final(out, detail_path(self.world))
                faulthandler.dump_traceback(all_threads=True)
                sys.stderr.flush()
                os._exit(held_rc)
            if self.rank == 0:
                out = base_line(self.args, self.world)
                out["error"] = "watchdog: phase '%s' overran its budget" % phase
                out["phase"] = phase
                parity = dict(self.parity)
                if transport is not None:
                    parity[transport] = False
                out["parity"] = parity
                emit(json.dumps(compact_line(out)))
            faulthandler.dump_traceback(all_threads=True)
            sys.stderr.flush()
            os._exit(3)


def injected(transport, rank, where):
    """DPWA_BENCH_INJECT="<transport>@<rank>[:start|:end|:die]" (test hook): raise inside that
    parity transport on that rank, at its start (before its first collective: the other ranks
    then block in one, and the watchdog ends the job) or at its end (after its rounds: the
    transport's isolation turns it into parity false); `die`: that rank exits at the transport's
    start (torch.distributed.run then stops the others with SIGTERM)."""
    spec = os.environ.get("DPWA_BENCH_INJECT", "")
    for item in filter(None, spec.split(",")):
        t, _, rest = item.partition("@")
        r, _, w = rest.partition(":")
        if t == transport and int(r or 0) == rank and (w or "end") == where:
            return True
    return False


class _NoCtxType:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NoCtx = _NoCtxType()


def write_config(path, names, interp, fetch_probability=1.0, divergence_threshold=0.0, self_peer=False,
                 base_port=45000):
    """The reference's YAML node config (dpwa/conn.py:246-262, dpwa/dpwa.py:60-90).  self_peer
    (configs[1], one learner): a second node entry "<name>-self" at the learner's own host:port --
    the reference's TxThread dials that address and reaches its own RxThread (conn.py:246-251 ->
    98-110), so the learner's peer is its own published snapshot."""
    if self_peer:
        names = [names[0], names[0] + "-self"]
    lines = ["- nodes:"] + ["  - {name: %s, host: 127.0.0.1, port: %d}" % (n, base_port + (0 if self_peer else i))
                            for i, n in enumerate(names)]
    lines += ["- fetch_probability: %r" % fetch_probability, "- timeout_ms: 2500",
              "- interpolation: %s" % interp, "- divergence_threshold: %r" % divergence_threshold,
              "- constant: { value: 0.5 }", "- clock: 0", "- loss: 0"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


# ---------------------------------------------------------------- CPU baselines (before the GPU)
def _timed(fn, seconds, min_rounds=1):
    rounds, t0 = 0, time.perf_counter()
    while True:
        fn()
        rounds += 1
        el = time.perf_counter() - t0
        if el >= seconds and rounds >= min_rounds:
            return rounds, el


def cpu_restatement_rows(seconds):
    """BASELINE.md CPU item 2: the averaging statement of pytorch.py:68 restated on the host at
    every north_star size -- numpy fp32 on one thread (a*t + b*p with f32 scalars, separately
    rounded; above NUMPY_SAMPLE_MAX elements on a bounded chunk of the workload) and torch-CPU
    eager in the config's dtype on every torch thread (fp32 also at 1B).  Reported like `value`:
    3*N*s averaged bytes per evaluation / time."""
    rows = []
    cores, threads = os.cpu_count(), torch.get_num_threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    g = torch.Generator().manual_seed(0)
    for numel, dt in SWEEP:
        esize = 4 if dt == "f32" else 2
        forms = [("torch_cpu", dt)] + ([("torch_cpu", "f32")] if dt == "bf16" and numel <= 1_000_000_000 else [])
        for kind, fdt in forms:
            tdtype = torch.float32 if fdt == "f32" else torch.bfloat16
            fs = 4 if fdt == "f32" else 2
            p = torch.empty(numel, dtype=tdtype).uniform_(-1.0, 1.0, generator=g)
            q = torch.empty(numel, dtype=tdtype).uniform_(-1.0, 1.0, generator=g)
            box = [p]

            def torch_round():
                box[0] = 0.5 * q + (1.0 - 0.5) * box[0]

            rounds, el = _timed(torch_round, seconds)
            rows.append({"numel": numel, "dtype": fdt, "config_dtype": dt, "kind": kind, "threads": threads,
                         "cpu_count": cores, "affinity_cpus": affinity, "rounds": rounds,
                         "ms_per_round": round(1e3 * el / rounds, 3),
                         "gbs": round(rounds * 3 * numel * fs / el / 1e9, 3),
                         "statement": "factor * t + (1 - factor) * p, torch eager (pytorch.py:68)"})
            del p, q, box
        m = min(numel, NUMPY_SAMPLE_MAX)
        pn = torch.empty(m, dtype=torch.float32).uniform_(-1.0, 1.0, generator=g).numpy()
        qn = torch.empty(m, dtype=torch.float32).uniform_(-1.0, 1.0, generator=g).numpy()
        a, b = np.float32(0.5), np.float32(1.0 - 0.5)
        pbox = [pn]

        def numpy_round():
            pbox[0] = a * qn + b * pbox[0]

        rounds, el = _timed(numpy_round, seconds)
        rows.append({"numel": numel, "dtype": "f32", "config_dtype": dt, "kind": "numpy_1thread", "threads": 1,
                     "cpu_count": cores, "affinity_cpus": affinity, "rounds": rounds,
                     "ms_per_round": round(1e3 * el / rounds * numel / m, 3),
                     "gbs": round(rounds * 3 * m * 4 / el / 1e9, 3),
                     "sample": ("whole vector" if m == numel else
                                "bounded: a %d-element chunk of the %d-element workload (rate is per byte; "
                                "ms_per_round scaled to the whole vector)" % (m, numel)),
                     "statement": "a * t + b * p, numpy float32, f32 scalars (restatement of pytorch.py:68)"})
        del pn, qn, pbox
        _ = esize
    return rows


def cpu_baseline(numel, seconds, rows=True):
    """The reference's CPU round (update_send -> TCP fetch -> update_wait; oracle/ref_round.py,
    which cites dpwa/adapters/pytorch.py, dpwa/conn.py and dpwa/messaging.py line by line)
    between two learner processes on this host, timed for ~`seconds`; reported like `value`
    (3*numel*4 averaged bytes per completed averaging).  Beside it, the C oracle running the
    same round's arithmetic on one host core (publish copy + averaging), and (rows) the
    averaging statement restated with numpy / torch-CPU at every north_star size."""
    from oracle import lerp as olerp
    from oracle import ref_round
    # one reference round at 100M fp32 already takes seconds: larger vectors are sampled
    out = ref_round.run(min(numel, REF_SAMPLE_MAX), seconds)
    if numel > REF_SAMPLE_MAX:
        out["sample"] += " (bounded sample of a %d-element workload)" % numel
    # BASELINE.md's second size: the same round at 100M fp32 (a few rounds; the reference's
    # 1B fp32 frame takes minutes per round and 1B/7B bf16 are not representable: N/A)
    out["rows"] = [ref_round.run(100_000_000, seconds / 2, min_rounds=3)] if numel != 100_000_000 else []
    out["rows_note"] = ("1B fp32: reference frame 4.0 GB, minutes per round (quadratic receive, messaging.py:55), not "
                        "sampled; 1B/7B bf16: not representable by the reference (pytorch.py:11-14, messaging.py:16)")
    ref_file = os.path.join(ROOT, "profiles", "reference_cpu_r02.json")
    if os.path.exists(ref_file):
        with open(ref_file) as f:
            ref = json.load(f)
        out["port_vs_reference"] = ref.get("port_vs_reference")
    lib = olerp.clib()
    rng = np.random.default_rng(0)
    param = rng.standard_normal(numel).astype(np.float32)
    peer = rng.standard_normal(numel).astype(np.float32)
    slot = np.empty_like(param)
    rounds = 0
    t0 = time.perf_counter()
    while True:
        lib.dpwa_oracle_publish(slot.ctypes.data, param.ctypes.data, param.nbytes)
        lib.dpwa_oracle_lerp_f32(param.ctypes.data, peer.ctypes.data, numel, 0.5)
        rounds += 1
        el = time.perf_counter() - t0
        if el >= seconds / 2:
            break
    out["c_oracle_round"] = {
        "value": rounds * 3 * numel * 4 / el / 1e9, "unit": "GB/s", "cores": 1, "cpu_count": os.cpu_count(),
        "sample": "%d rounds of publish-copy + fp32 lerp over %d elements (oracle/dpwa_oracle.c, -O3, 1 thread, "
                  "%.1f s): the arithmetic alone, no transport" % (rounds, numel, el),
        "ms_per_round": 1e3 * el / rounds}
    # and the reference's own lerp statement (pytorch.py:68, torch eager) on every thread torch
    # uses here: the multi-core CPU ceiling for the arithmetic
    tp, tq = torch.from_numpy(param), torch.from_numpy(peer)
    rounds = 0
    t0 = time.perf_counter()
    while True:
        tp = 0.5 * tq + (1.0 - 0.5) * tp
        rounds += 1
        el = time.perf_counter() - t0
        if el >= min(3.0, seconds / 3):
            break
    out["torch_cpu_lerp"] = {
        "value": rounds * 3 * numel * 4 / el / 1e9, "unit": "GB/s", "cores": torch.get_num_threads(),
        "threads": torch.get_num_threads(), "cpu_count": os.cpu_count(),
        "sample": "%d evaluations of the reference's lerp statement (pytorch.py:68) as torch-CPU fp32 eager ops "
                  "over %d elements, %.1f s" % (rounds, numel, el),
        "ms_per_round": 1e3 * el / rounds}
    del param, peer, slot, tp, tq
    if rows:
        out["restatement_rows"] = cpu_restatement_rows(max(1.0, seconds / 8))
        out["restatement_note"] = ("BASELINE.md CPU item 2: numpy fp32 one thread, torch-CPU in the config dtype "
                                   "(and fp32 to 1B) on every torch thread, at 11.17M / 100M / 1B / 7B; "
                                   "cpu_count = os.cpu_count(), threads = torch.get_num_threads()")
    return out


# ---------------------------------------------------------------- parity leg (checker)
# A short deterministic gossip through every transport the run uses, checked bit for bit
# against the oracle (oracle/ is imported only here and by the cpu_baseline leg, as the
# checker -- never on the measured path).
PARITY_N, PARITY_T, PARITY_FP = 1_000_003, 12, 0.7
OVERLAP_PAIRS = 4               # interleaved (step alone, step + gossip) pairs of the overlap leg
PARITY_ASYNC_T = 16
PARITY_PHASE_S = 180.0          # watchdog budget of one parity transport


def parity_transports(world, gossip="auto"):
    """Every transport the run can time, plus the fd-shared (hipMemCreate, DPWA_VMM=1) slot
    path that configs[3]/[4] use above 1.5 GiB, through the lock-step fused relay (slots and
    relay buffers fd-imported) and the free-running board.  main() checks the `+vmm` ones at N>1
    only after the measured line is held (no timed transport uses them)."""
    if world == 1:
        return ["self", "local", "local+res"]
    t = []
    if gossip != "async":
        t += ["lockstep/copy", "lockstep/kernel:256", "lockstep/relay:32", "lockstep/relay-avg:32",
              "lockstep/relay-avg:32+vmm", "lockstep/copy+res", "lockstep/kernel:256+res", "lockstep/relay:32+res",
              "lockstep/relay-avg:32+res", "lockstep/relay-avg:32+res+vmm"]
    if gossip != "lockstep":
        t += ["async/copy", "async/kernel:256", "async/copy+wt", "async/kernel:256+wt", "async/copy+vmm",
              "async/copy+res", "async/kernel:256+res", "async/copy+res+vmm"]
    return t


def parity_init(g, n):
    return np.random.default_rng([31, g]).standard_normal(n).astype(np.float32)


def parity_delta(g, r, n):
    return (0.01 * np.random.default_rng([32, r, g]).standard_normal(n)).astype(np.float32)


def parity_loss(g, r, wait):
    x = 2.0 * float(np.exp(-r / 4.0)) + 0.01 * g + 0.003
    return 0.95 * x if wait else x


def parity_lockstep(names, mine, cfg, group, pull, device, n=PARITY_N, T=PARITY_T, conns=None, batch=False,
                    resident=False):
    """T lock-step rounds (clock interpolation, fetch_probability PARITY_FP) of the learners
    `mine` = [(name, g)] through the drop-in API: the training step adds a seeded delta; two
    of three rounds average with the fused kernel and write-through snapshots (the adapter's
    default; with `batch`, all of this process's learners in one dispatch), every third through
    the split update_wait + average.  `resident`: the parameters live in the learners' slots
    (make_resident), every round averages fused (batched with `batch`) and the training step
    comes after update_wait, as a resident loop must run.  Returns per learner g the per-round
    (sha1 of the parameters after the average, clock, peer averaged with).  `conns` (a list)
    receives the connections as they are made, so a caller can close them after a failure."""
    import hashlib
    from dpwa_amd import DpwaConnection
    conns = [] if conns is None else conns
    flats = []
    for name, g in mine:
        conns.append(DpwaConnection(name, cfg, seed=900 + g, group=group, pull=pull))
        flats.append(torch.from_numpy(parity_init(g, n)).to(device))
    if resident:
        return conns, _parity_lockstep_resident(conns, flats, mine, device, n, T, batch)
    rec = {g: [] for _, g in mine}
    for r in range(T):
        wt_prev = r % 3 != 0        # the previous round averaged write-through (r % 3 == 2 is split)
        for conn, flat, (_, g) in zip(conns, flats, mine):
            conn.update_send(flat, parity_loss(g, r, False), reuse_snapshot=wt_prev and r > 0)
        for flat, (_, g) in zip(flats, mine):
            flat.add_(torch.from_numpy(parity_delta(g, r, n)).to(device))
        got = []
        if r % 3 != 2 and batch:
            res = DpwaConnection.update_wait_average_many(conns, flats, [parity_loss(g, r, True) for _, g in mine],
                                                          write_through=True)
            got = [p.peer if p is not None else "" for p, _ in res]
        else:
            for conn, flat, (_, g) in zip(conns, flats, mine):
                if r % 3 == 2:
                    payload, factor = conn.update_wait(parity_loss(g, r, True))
                    if payload is not None:
                        conn.average(flat)
                else:
                    payload, _ = conn.update_wait_average(flat, parity_loss(g, r, True), write_through=True)
                got.append(payload.peer if payload is not None else "")
        for conn, flat, (_, g), peer in zip(conns, flats, mine, got):
            rec[g].append((hashlib.sha1(flat.cpu().numpy().tobytes()).hexdigest(), conn.clock, peer))
    torch.cuda.synchronize()
    return conns, rec


def _parity_lockstep_resident(conns, flats, mine, device, n, T, batch):
    import hashlib
    from dpwa_amd import DpwaConnection
    for conn, flat in zip(conns, flats):
        conn.make_resident(flat)
    rec = {g: [] for _, g in mine}
    for r in range(T):
        for conn, (_, g) in zip(conns, mine):
            conn.update_send(conn.parameters, parity_loss(g, r, False))
        if batch:
            res = DpwaConnection.update_wait_average_many(conns, [c.parameters for c in conns],
                                                          [parity_loss(g, r, True) for _, g in mine])
        else:
            res = [conn.update_wait_average(conn.parameters, parity_loss(g, r, True)) for conn, (_, g) in zip(conns, mine)]
        for conn, (_, g), (p, _) in zip(conns, mine, res):
            rec[g].append((hashlib.sha1(conn.parameters.cpu().numpy().tobytes()).hexdigest(), conn.clock,
                           p.peer if p is not None else ""))
        for conn, (_, g) in zip(conns, mine):      # the training step, after update_wait
            conn.parameters.add_(torch.from_numpy(parity_delta(g, r, n)).to(device))
    torch.cuda.synchronize()
    return rec


def parity_self(cfg, device, n=PARITY_N, T=PARITY_T, conns=None):
    """The N=1 timed form: one learner whose peer is its own snapshot (a self-peer config), T rounds
    in the reference order -- update_send (reusing the snapshot the last average wrote through),
    the seeded training delta, update_wait_average with the write-through average -- clock
    interpolation, fetch_probability PARITY_FP.  Returns the per-round (sha1 of the parameters,
    clock, peer)."""
    import hashlib
    from dpwa_amd import DpwaConnection
    from dpwa_amd.group import LocalGroup
    conns = [] if conns is None else conns
    conn = DpwaConnection("w1", cfg, seed=900, group=LocalGroup())
    conns.append(conn)
    flat = torch.from_numpy(parity_init(0, n)).to(device)
    rec, reuse = [], False
    for r in range(T):
        conn.update_send(flat, parity_loss(0, r, False), reuse_snapshot=reuse)
        flat.add_(torch.from_numpy(parity_delta(0, r, n)).to(device))
        payload, _ = conn.update_wait_average(flat, parity_loss(0, r, True), write_through=True)
        reuse = payload is not None
        rec.append((hashlib.sha1(flat.cpu().numpy().tobytes()).hexdigest(), conn.clock,
                    payload.peer if payload is not None else ""))
    torch.cuda.synchronize()
    return rec


def parity_self_expected(n=PARITY_N, T=PARITY_T):
    """oracle/gossip.py's trajectory of parity_self: nodes [w1, w1-self], w1-self served by w1
    (pinned to the reference's own self-peer runs, tests/golden/gossip_self.*)."""
    import hashlib
    from oracle import gossip as ogossip
    init = parity_init(0, n)[None]
    deltas = np.stack([parity_delta(0, r, n)[None] for r in range(T)])
    exp = ogossip.simulate(["w1"], init, deltas, [[parity_loss(0, r, False)] for r in range(T)],
                           [[parity_loss(0, r, True)] for r in range(T)], "clock", None, 0.0, PARITY_FP, [900],
                           nodes=["w1", "w1-self"], serves={"w1-self": 0})
    return [(hashlib.sha1(exp["params"][r, 0].tobytes()).hexdigest(), float(exp["clocks"][r, 0]),
             (exp["picks"][r][0][-1] if exp["picks"][r][0] else "")) for r in range(T)]


def parity_lockstep_expected(names, n=PARITY_N, T=PARITY_T, resident=False):
    """The oracle's trajectory of parity_lockstep (oracle/gossip.py, pinned to the reference)."""
    import hashlib
    from oracle import gossip as ogossip
    G = len(names)
    init = np.stack([parity_init(g, n) for g in range(G)])
    deltas = np.stack([np.stack([parity_delta(g, r, n) for g in range(G)]) for r in range(T)])
    send = [[parity_loss(g, r, False) for g in range(G)] for r in range(T)]
    wait = [[parity_loss(g, r, True) for g in range(G)] for r in range(T)]
    exp = ogossip.simulate(names, init, deltas, send, wait, "clock", None, 0.0, PARITY_FP,
                           [900 + g for g in range(G)], train_after_wait=resident)
    return {g: [(hashlib.sha1(exp["params"][r, g].tobytes()).hexdigest(), float(exp["clocks"][r, g]),
                 (exp["picks"][r][g][-1] if exp["picks"][r][g] else ""))
                for r in range(T)] for g in range(G)}


def parity_async(names, rank, cfg, pull, device, n=PARITY_N, T=PARITY_ASYNC_T, write_through=False, conns=None,
                 resident=False):
    """Free-running rounds over the gossip board (AsyncDistGroup): each round publishes, runs
    an uneven synthetic step that sets the parameters to the checker's known values for
    (rank, round) and averages with whatever version the board hands out.  Without
    write-through the publish comes after that step (it publishes the known values); with it,
    before (it publishes what the last average wrote through).  `resident`: the parameters live
    in the learner's slots; the step sets them after the average (before the next publish, as
    a resident loop must), so the publish carries the known values as without write-through.
    Returns (params, clocks, peers, versions)."""
    from dpwa_amd import DpwaConnection
    from oracle.async_check import async_base, async_loss
    conn = DpwaConnection(names[rank], cfg, seed=700 + rank, group="async", pull=pull)
    if conns is not None:
        conns.append(conn)
    rng = np.random.default_rng(rank)
    flat = torch.from_numpy(async_base(rank, -1, n)).to(device)
    bases = [torch.from_numpy(async_base(rank, r, n)).to(device) for r in range(T)]
    params, clocks, peers, versions = np.zeros((T, n), np.float32), np.zeros(T), [], []
    if resident:
        conn.make_resident(flat)
        for r in range(T):
            conn.parameters.copy_(bases[r])
            conn.update_send(conn.parameters, async_loss(rank, r))
            torch.cuda._sleep(int(rng.integers(0, 200_000)))   # uneven "training steps" (nothing written)
            payload, _ = conn.update_wait_average(conn.parameters, async_loss(rank, r, wait=True))
            peers.append(payload.peer if payload is not None else "")
            versions.append(conn._info()[2] if payload is not None else 0)
            params[r] = conn.parameters.cpu().numpy()
            clocks[r] = conn.clock
        torch.cuda.synchronize()
        return params, clocks, peers, versions
    for r in range(T):
        if not write_through:
            flat.copy_(bases[r])
        conn.update_send(flat, async_loss(rank, r), reuse_snapshot=write_through)
        if write_through:
            flat.copy_(bases[r])
        torch.cuda._sleep(int(rng.integers(0, 200_000)))       # uneven "training steps"
        payload, _ = conn.update_wait_average(flat, async_loss(rank, r, wait=True), write_through=write_through)
        peers.append(payload.peer if payload is not None else "")
        versions.append(conn._info()[2] if payload is not None else 0)
        params[r] = flat.cpu().numpy()
        clocks[r] = conn.clock
    torch.cuda.synchronize()
    return params, clocks, peers, versions


def parity_key(trial):
    """The parity transport that vouches for a transport trial key ("<mode>[+res]" lock-step or
    "async/<mode>[+wt|+res]"): kernel pulls of any grid and relays of any block count share the
    kernels of the parity run's kernel:256 / relay:32."""
    kind, _, mode = trial.rpartition("/")
    form = "+wt" if mode.endswith("+wt") else "+res" if mode.endswith("+res") else ""
    base = trial_mode(mode).partition(":")[0]
    pull = {"copy": "copy", "kernel": "kernel:256", "relay": "relay:32", "relay-avg": "relay-avg:32"}[base]
    return "%s/%s%s" % (kind or "lockstep", pull, form)


TRAFFIC_ROUNDS = ("r06", "r05", "r04", "r03")     # profiles/traffic_<round>_<publish>[_x<learners>].json, newest first


def pmc_traffic(path, publish, learners, numel, dtype, basis):
    """(HBM bytes per launch, source) of a kernel from a committed PMC summary (tools/pmc_traffic.py
    over rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/cold_sweep.py), if one matches this
    workload; else (None, None)."""
    name = "%s%s.json" % (publish, "_x%d" % learners if learners > 1 else "")
    paths = [path] if path else [os.path.join(ROOT, "profiles", "traffic_%s_%s" % (r, name)) for r in TRAFFIC_ROUNDS]
    for tpath in paths:
        if not os.path.exists(tpath):
            continue
        with open(tpath) as f:
            tr = json.load(f)
        if (tr.get("numel") == numel and tr.get("dtype") == dtype and tr.get("publish", "full") == publish and
                tr.get("learners_per_launch", 1) == learners and tr.get("basis", "in-loop") == basis):
            return tr.get("hbm_bytes_per_launch"), os.path.relpath(tpath, ROOT)
    return None, None


def write_through_key(world, chosen):
    """The parity transport that vouches for the write-through learners a resident run times
    beside its own (secondary_publish, reference_loop, overlap): the chosen trial's pull in the
    write-through form ("local" at N=1)."""
    if world == 1:
        return "local"
    mode = trial_mode(chosen)
    return parity_key(("async/" + mode + "+wt") if chosen.startswith("async/") else mode)


def trial_mode(key):
    """The pull mode of a trial key: "async/copy+wt" -> "copy", "relay-avg:32+res" -> "relay-avg:32"."""
    return key.split("/")[-1].replace("+wt", "").replace("+res", "")


class _Env:
    """Sets environment variables for the duration of a with-block (DPWA_VMM for +vmm)."""

    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def provisional_line(args, world, rank, device, cfg, mine, dtype, ctl, watchdog, parity):
    """N>1 insurance for the driver's multi-GPU run: right after `lockstep/copy` (the plainest
    transport: a copy-engine pull from an IPC-mapped slot) passed its parity check, the line's
    rounds are timed once on it -- --warmup untimed and --steps timed lock-step rounds,
    write-through, barrier + synchronize on both sides, max over ranks -- before any other
    transport runs on this node's devices.  Rank 0 gets the provisional line (the others None);
    main() holds it, so a hang, a fault or a stop in what follows still leaves a verified,
    measured line (marked `provisional`).  The learners are closed before the parity leg goes on.
    Returns (ok, line): ok agreed over the ranks; line on rank 0 only."""
    from dpwa_amd import DpwaConnection
    watchdog.enter("provisional measurement (lockstep/copy)", 300.0)
    esize = 4 if dtype == torch.float32 else 2
    conns, err, el, averaged = [], None, None, 0
    try:
        for name, seed in mine:
            g = torch.Generator(device=device).manual_seed(seed)
            flat = torch.randn(args.numel, device=device, generator=g, dtype=torch.float32).to(dtype)
            conns.append((DpwaConnection(name, cfg, seed=1000 + seed, group="lockstep", pull="copy"), flat))

        def step():
            done = 0
            for conn, flat in conns:
                conn.update_send(flat, 1.0, reuse_snapshot=True)
            for conn, flat in conns:
                done += conn.update_wait_average(flat, 1.0, write_through=True)[0] is not None
            return done

        for _ in range(max(1, args.warmup)):
            step()
        torch.cuda.synchronize()
        dist.barrier(group=ctl)
        t0 = time.perf_counter()
        averaged = sum(step() for _ in range(args.steps))
        torch.cuda.synchronize()
        dist.barrier(group=ctl)
        el = time.perf_counter() - t0
    except Exception as e:   # noqa: BLE001 -- no provisional line; the run goes on as before
        err = "%s: %s" % (type(e).__name__, e)
        progress("provisional measurement FAILED: %s" % err)
    finally:
        for conn, _ in conns:
            try:
                conn.close()
            except Exception as e:   # noqa: BLE001
                progress("provisional close: %s" % e)
        conns = []
        torch.cuda.synchronize()
    ok = _agree(err is None, world, ctl)
    got = [None] * world
    dist.all_gather_object(got, (el, averaged), group=ctl)
    dist.barrier(group=ctl)
    watchdog.idle()
    if not ok or rank != 0:
        return ok, None
    el_max = max(g[0] for g in got)
    av = sum(g[1] for g in got)
    out = base_line(args, world)
    value = round(av * 3 * args.numel * esize / el_max / 1e9, 2)
    rps = round(world * args.steps / el_max, 1)
    out.update({
        "value": value,
        "ms_per_step": round(1e3 * el_max / args.steps, 4),
        "gossip_rounds_per_s": rps,
        "averagings": int(av),
        "provisional": True,
        # the kernel is not timed on its own in this pass: the roofline block names it and its bytes
        "roofline": {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                     "traffic": None, "bytes_per_launch": 4 * args.numel * esize, "avg_launch_us": None,
                     "metric_bytes_per_averaging": 3 * args.numel * esize,
                     "kernel": "dpwa::k_lerp<Ops%s, COEF_FUSED, true> (not timed alone in the provisional pass)"
                               % args.dtype.upper()},
        "scaling_basis": {"n_gpus": world, "learners_per_gpu": len(mine), "publish": "write-through",
                          "raw": {"gossip_rounds_per_s": rps, "value": value}, "weak": {}},
        "config": {"workload": "north_star on-node gossip, one learner per GPU (provisional: lockstep/copy)",
                   "numel": args.numel, "pull": "lockstep/copy", "publish": "write-through",
                   "interpolation": args.interpolation, "fetch_probability": args.fetch_probability,
                   "learners_per_gpu": len(mine)},
        "parity": parity,
        "parity_of_timed_transport": {"transport": "lockstep/copy", "ok": True},
        "note": "measured before the other transports were checked and timed, so that the line survives them",
    })
    progress("provisional: %.1f GB/s (%.4f ms/step)" % (out["value"], out["ms_per_step"]))
    return ok, out


def parity_leg(world, rank, local_rank, device, cfg_dir, transports, dist_backend, ctl=None, watchdog=None):
    """Runs the parity workload through `transports` and returns {transport: bool} on every
    rank (rank 0 compares the lock-step digests with the oracle; each rank checks its own
    free-running rounds).  Each transport is isolated: an exception on any rank becomes that
    transport's `false` (the ranks agree over `ctl`, a gloo group, in the same collectives
    whatever happened), and its connections are closed before the next one starts.  A hang
    inside a transport is the watchdog's."""
    names = ["w%d" % (g + 1) for g in range(max(world, 2))]
    cfg = os.path.join(cfg_dir, "parity.yaml")
    write_config(cfg, names, "clock", PARITY_FP, 0.0)
    cfg_self = os.path.join(cfg_dir, "parity_self.yaml")
    write_config(cfg_self, ["w1"], "clock", PARITY_FP, 0.0, self_peer=True, base_port=45900)
    if world > 1 and ctl is None:
        ctl = dist.new_group(backend="gloo")
    result = {}
    expected = ({False: parity_lockstep_expected(names), True: parity_lockstep_expected(names, resident=True)}
                if rank == 0 else None)
    for t in transports:
        if watchdog is not None:
            watchdog.enter("parity %s" % t, PARITY_PHASE_S, transport=t)
        else:
            progress("parity %s" % t)
        kind, _, pull = t.partition("/")
        vmm = pull.endswith("+vmm")
        pull = pull.replace("+vmm", "")
        res = kind.endswith("+res") or pull.endswith("+res")
        kind, pull = kind.replace("+res", ""), pull.replace("+res", "")
        conns, err, rec, check = [], None, None, None
        try:
            with _Env(DPWA_VMM="1") if vmm else _Env():
                if injected(t, rank, "die"):
                    progress("injected exit (DPWA_BENCH_INJECT, die)")
                    os._exit(7)
                if injected(t, rank, "start"):
                    raise RuntimeError("injected failure (DPWA_BENCH_INJECT, start)")
                if kind == "self":                    # the N=1 timed form: one learner, its own snapshot
                    rec = parity_self(cfg_self, device, conns=conns)
                elif kind == "local":                 # one GPU: both learners in this process, batched
                    from dpwa_amd.group import LocalGroup
                    _, rec = parity_lockstep(names, [(names[0], 0), (names[1], 1)], cfg, LocalGroup(), None, device,
                                             conns=conns, batch=True, resident=res)
                elif kind == "lockstep":
                    _, r = parity_lockstep(names, [(names[rank], rank)], cfg, "lockstep", pull, device, conns=conns,
                                           resident=res)
                    rec = r[rank]
                else:                                  # async: free-running over the gossip board
                    wt = pull.endswith("+wt")
                    check = parity_async(names, rank, cfg, pull.replace("+wt", ""), device, write_through=wt,
                                         conns=conns, resident=res)
                if injected(t, rank, "end"):
                    raise RuntimeError("injected failure (DPWA_BENCH_INJECT, end)")
        except Exception as e:   # noqa: BLE001 -- reported as this transport's parity false
            err = "%s: %s" % (type(e).__name__, e)
            progress("parity %s FAILED on rank %d: %s" % (t, rank, err))
        finally:
            for c in conns:
                try:
                    c.close()
                except Exception as e:   # noqa: BLE001
                    progress("parity %s: close failed: %s" % (t, e))
        want = expected[res] if expected is not None else None
        if kind == "self":
            ok = err is None and rec == parity_self_expected()
        elif kind == "local":
            ok = err is None and rec == want
        elif kind == "lockstep":
            got = [None] * world
            dist.all_gather_object(got, rec if err is None else None, group=ctl)
            ok = rank != 0 or (all(g is not None for g in got) and all(got[g] == want[g] for g in range(world)))
        else:
            ok = _async_verdict(t, names, world, rank, check, err, ctl)
        if err is not None:
            ok = False
        result[t] = bool(_agree(ok, world, ctl) if world > 1 else ok)
        if watchdog is not None:
            watchdog.parity[t] = result[t]
        try:
            torch.cuda.synchronize()
        except Exception as e:   # noqa: BLE001
            progress("parity %s: synchronize failed: %s" % (t, e))
        if world > 1:
            dist.barrier(group=ctl)
    if watchdog is not None:
        watchdog.idle()
    return result


def _agree(ok, world, ctl):
    """All ranks' verdicts, AND-ed, on every rank (a gloo all_gather: the CPU control group)."""
    if world <= 1:
        return bool(ok)
    got = [None] * world
    dist.all_gather_object(got, bool(ok), group=ctl)
    return all(got)


def _async_verdict(t, names, world, rank, check, err, ctl):
    """Free-running rounds: every rank checks its own rounds version by version against
    oracle/async_check.py; the (peers, versions) of every rank are gathered first (every rank
    enters the same collectives whether or not its run failed)."""
    from oracle.async_check import AsyncRuns, async_base
    wt = t.endswith("+wt")
    got = [None] * world
    dist.all_gather_object(got, (check[2], check[3]) if check is not None else None, group=ctl)
    if any(g is None for g in got):     # every rank sees it: none enters the next collective
        return False
    params, clocks = check[0], check[1]
    runs = AsyncRuns(names, {g: got[g][0] for g in range(world)}, {g: got[g][1] for g in range(world)},
                     "clock", None, 0.0)
    if wt:   # each rank vouches for the averages of its own published versions (digests)
        mine = runs.served(rank, lambda v: async_base(rank, -1, PARITY_N) if v == 1 else params[v - 2], PARITY_N)
        served = [None] * world
        dist.all_gather_object(served, mine, group=ctl)
        vouched = {}
        for d in served:
            vouched.update(d)
        bad = runs.check_rank_digests(rank, params, clocks, PARITY_N, vouched)
    else:
        bad = runs.check_rank(rank, params, clocks, PARITY_N)
    if bad:
        print("parity %s rank %d: %s" % (t, rank, bad[:3]), file=sys.stderr, flush=True)
    return not bad


# ---------------------------------------------------------------- kernel measurements
def cold_kernel(numel, dtype, device, write_through=False, launches=64, learners=1, resident=False, pair=False,
                mix=False):
    """The product averaging kernel alone over rotating buffers (> 1.2 GB of other traffic
    between two uses of a buffer, so nothing is served from the 256 MiB Infinity Cache).  With
    learners == 1 it is dpwa_average (k_lerp<Ops, COEF_FUSED, write_through>: fp64 device
    factor + lerp in place, with write_through the result also stored into a snapshot
    payload); with learners > 1, dpwa_average_many: that many independent averages in ONE
    dispatch (k_lerp_batch, the N=1 loop's kernel).  Every launch is timed by its own dispatch
    begin/end events (hipExtLaunchKernelGGL), as rocprofv3 times a kernel: the inter-kernel
    gaps of a back-to-back batch are not counted.  Also returns the rate of one event pair
    around the whole batch (which does include the gaps).  `resident`: the resident form
    (dpwa_average_many_resident): the parameters are read from one snapshot payload and the result
    stored into another, nothing written back in place (3*N*s).  `pair` (resident, 2 learners): the
    two learners average with each other, as the N=1 loop's do -- entry 0 reads A's slot and B's,
    entry 1 B's and A's -- so the dispatch is a mutual pair (k_lerp_pair: 4*N*s).
    `mix` (one learner, in place): every product launch is followed by one of its access mix alone
    (dpwa_stream_mix: the same loads and stores, same addresses -- the parameters and the peer
    payload read, the parameters and the snapshot written -- same launch shape and cache policy,
    no factor, no lerp) over another set of the same rotation, each timed by its own dispatch
    events: the ceiling of that mix measured interleaved with the product kernel, on its buffers,
    returned under "mix"."""
    from dpwa_amd import _lib
    esize = 4 if dtype == torch.float32 else 2
    write_through = write_through or resident
    pair = pair and resident and learners == 2
    nbuf = 3 if write_through else 2
    per_set = (4 if pair else learners * nbuf) * numel * esize
    # > 1.2 GB of other traffic between two uses of a buffer; a set that large by itself is its
    # own rotation (7B bf16: 42 GB per learner, HBM holds the learners' slots too)
    sets = 1 if per_set >= 1.2e9 else max(2, int(np.ceil(1.2e9 / per_set)))
    # at least 4 timed launches (a 1B / 7B launch is 1-9 ms: one slow launch of two moved a mean by 50 %)
    launches = max(2 * sets, 4, min(launches, int(np.ceil(64 * 134e6 / (3 * learners * numel * esize)))))
    hdr = _lib.SLOT_PAYLOAD_OFFSET // esize
    bufs = []       # per set: [(param, slot, snap)] * learners
    for _ in range(sets):
        entries = []
        if pair:    # two published slots, each the parameters of one learner and the peer of the other
            slots = [torch.zeros(hdr + numel, device=device, dtype=dtype) for _ in range(2)]
            for sl in slots:
                sl[hdr:].normal_()
            nxt = [torch.empty(hdr + numel, device=device, dtype=dtype)[hdr:] for _ in range(2)]
            entries = [(slots[0][hdr:], slots[1], nxt[0]), (slots[1][hdr:], slots[0], nxt[1])]
        for _ in range(0 if pair else learners):
            param = torch.empty(numel, device=device, dtype=dtype).normal_()
            # a snapshot slot as the learner lays it out: header (zeros) and pad, then the payload
            slot = torch.zeros(hdr + numel, device=device, dtype=dtype)
            slot[hdr:].normal_()
            # the write-through destination is the payload of another slot
            snap = torch.empty(hdr + numel, device=device, dtype=dtype)[hdr:] if write_through else None
            entries.append((param, slot, snap))
        bufs.append(entries)
    clocks = torch.zeros(learners, 2, device=device, dtype=torch.float64)
    coefs = torch.zeros(learners, 4, device=device, dtype=torch.float64)           # dpwa_coef, 32 B
    cfg = _lib.Interp(_lib.INTERP_CONSTANT, 0, 0.5, 0.0)
    dt = _lib.F32 if dtype == torch.float32 else _lib.BF16
    s = _lib.stream_handle(None)
    lib = _lib.load()
    descs = []
    for entries in bufs:
        d = (_lib.AverageDesc * learners)()
        for j, (param, slot, snap) in enumerate(entries):
            d[j] = _lib.AverageDesc(param.data_ptr(), slot.data_ptr(), numel, clocks[j].data_ptr(), 1.0,
                                    coefs[j].data_ptr(), snap.data_ptr() if snap is not None else None)
        descs.append(d)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    for a, b in ev:          # create the events (the kernel dispatch then records into them)
        a.record()
        b.record()

    def run(i, timed):
        a, b = ev[i] if timed else (None, None)
        ea, eb = (a.cuda_event, b.cuda_event) if timed else (None, None)
        if resident:
            rc = lib.dpwa_average_many_resident(dt, descs[i % sets], learners, ctypes.byref(cfg), s, ea, eb)
            name = "dpwa_average_many_resident"
        elif learners == 1:
            param, slot, snap = bufs[i % sets][0]
            rc = lib.dpwa_average(dt, param.data_ptr(), slot.data_ptr(), numel, ctypes.byref(cfg),
                                  clocks[0].data_ptr(), 1.0, coefs[0].data_ptr(),
                                  snap.data_ptr() if snap is not None else None, s, ea, eb)
            name = "dpwa_average"
        else:
            rc = lib.dpwa_average_many(dt, descs[i % sets], learners, ctypes.byref(cfg), s, ea, eb)
            name = "dpwa_average_many"
        if rc:
            raise _lib.DpwaError(name, rc, lib.dpwa_last_error().decode())

    mix = mix and learners == 1 and not resident
    nbytes = numel * esize // 16 * 16
    if mix:
        evm = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
        for a, b in evm:
            a.record()
            b.record()
        mix_ptrs = []
        for entries in bufs:
            param, slot, snap = entries[0]
            dst = [param.data_ptr()] + ([snap.data_ptr()] if snap is not None else [])
            mix_ptrs.append(((ctypes.c_void_p * 2)(*dst), (ctypes.c_void_p * 2)(slot[hdr:].data_ptr(), param.data_ptr()),
                             len(dst)))

    def run_mix(i):
        dst, src, nw = mix_ptrs[(i + sets // 2) % sets]     # half a rotation away from the product launch
        rc = lib.dpwa_stream_mix(dst, nw, src, 2, nbytes, s, evm[i][0].cuda_event, evm[i][1].cuda_event)
        if rc:
            raise _lib.DpwaError("dpwa_stream_mix", rc, lib.dpwa_last_error().decode())

    for i in range(sets):
        run(i, False)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(50_000_000)          # let the host queue the whole batch first
    t0.record()
    for i in range(launches):
        run(i, True)
        if mix:
            run_mix(i)
    t1.record()
    torch.cuda.synchronize()
    us = np.array([a.elapsed_time(b) * 1e3 for a, b in ev])
    batch_us = t0.elapsed_time(t1) * 1e3 / launches
    out = {"avg_launch_us": float(us.mean()), "median_launch_us": float(np.median(us)),
           "min_launch_us": float(us.min()), "max_launch_us": float(us.max()), "launches": launches,
           "rotating_buffer_sets": sets, "learners_per_launch": learners, "batch_bracket_us": float(batch_us),
           "mutual_pair": pair}
    if mix:
        um = np.array([a.elapsed_time(b) * 1e3 for a, b in evm])
        nw = mix_ptrs[0][2]
        moved = (2 + nw) * nbytes
        gbs = moved / (float(um.mean()) * 1e-6) / 1e9
        out["mix"] = {"mix": "2R:%dW" % nw, "bytes_per_launch": moved, "avg_launch_us": round(float(um.mean()), 2),
                      "median_launch_us": round(float(np.median(um)), 2), "achieved": round(gbs, 1),
                      "frac": round(gbs / HBM_PEAK_GBS, 4), "launches": launches, "rotating_buffer_sets": sets,
                      "interleaved": True, "kernel": "dpwa::k_stream_mix<2, %d> (dpwa_stream_mix)" % nw}
    del bufs, descs
    torch.cuda.empty_cache()
    return out


def round_sweep(device, cfg_dir, steps=20, warmup=3, rows=None, publish="write-through", min_s=0.25):
    """Whole gossip rounds of the N=1 line's form at every north_star size in its config's dtype:
    one learner whose peer is its own snapshot (configs[1]'s self-peer), constant 0.5,
    fetch_probability 1, `publish` write-through (the snapshot the average writes through is the
    next publish) or full (every publish copies the 2*N*s snapshot) -- the averaged GB/s and
    rounds/s the north star asks for at 11M/100M/1B/7B on one GPU, on the basis of the N>1 sweep
    (one learner per GPU).  Each size runs at least `steps` rounds and at least `min_s` seconds
    (sized from one probe round)."""
    from dpwa_amd import DpwaConnection
    from dpwa_amd.group import LocalGroup
    rows = [] if rows is None else rows
    cfg = os.path.join(cfg_dir, "sweep.yaml")
    write_config(cfg, ["w1"], "constant", self_peer=True, base_port=45800)
    wt = publish == "write-through"
    for numel, dt in SWEEP:
        dtype = torch.float32 if dt == "f32" else torch.bfloat16
        esize = 4 if dt == "f32" else 2
        flat = torch.empty(numel, dtype=dtype, device=device)
        flat.normal_(generator=torch.Generator(device=device).manual_seed(0))
        conn = DpwaConnection("w1", cfg, seed=1000, group=LocalGroup())

        def step():
            conn.update_send(flat, 1.0, reuse_snapshot=wt)
            return conn.update_wait_average(flat, 1.0, write_through=wt)[0] is not None

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()       # one more round sizes the timed run: >= min_s, at least `steps`
        step()
        torch.cuda.synchronize()
        n_steps = int(max(steps, min(20000, np.ceil(min_s / max(time.perf_counter() - t0, 1e-6)))))
        t0 = time.perf_counter()
        averaged = sum(step() for _ in range(n_steps))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rows.append({"numel": numel, "dtype": dt, "value": round(averaged * 3 * numel * esize / el / 1e9, 1),
                     "ms_per_step": round(1e3 * el / n_steps, 4), "gossip_rounds_per_s": round(n_steps / el, 1),
                     "steps": n_steps, "seconds": round(el, 3), "learners": 1, "peer": "self", "publish": publish})
        conn.close()
        del flat, conn
        torch.cuda.empty_cache()
    return rows


VMM_MIN_BYTES = 3 << 29     # learner.cpp kVmmMinBytes: slots from here up are fd-shared hipMemCreate chunks


def dist_round_sweep(world, rank, device, cfg_dir, pull, write_through, ctl, watchdog, min_steps=3, warmup=2,
                     max_numel=None, rows=None, resident=False, vmm_ok=True):
    """N > 1: whole gossip rounds at every north_star size (configs[1..4] sizes and dtypes), one
    learner per rank, on the transport the trials chose (`pull`: "<mode>" lock-step or
    "async/<mode>[+wt]"), constant 0.5, fetch_probability 1 -- the GB/s and rounds/s table of
    BASELINE's north_star at 2/4/8 GPUs.  A size that fails on any rank is reported with its
    error and the sweep goes on.  max_numel: skip larger sizes (rehearsals with several ranks
    on one GPU).  vmm_ok False (a `+vmm` parity transport failed on this node's devices): the
    sizes whose slots would be fd-shared hipMemCreate chunks are reported as not run instead of
    mapping memory that failed its check."""
    from dpwa_amd import DpwaConnection
    names = ["w%d" % (r + 1) for r in range(world)]
    cfg = os.path.join(cfg_dir, "dist_sweep.yaml")     # every rank its own copy (cfg_dir is per rank)
    write_config(cfg, names, "constant")
    sel_async = pull.startswith("async/")
    mode = trial_mode(pull)
    # ranks sharing a device (rehearsals) split its free memory
    share = max(1, -(-world // max(1, torch.cuda.device_count())))
    rows = [] if rows is None else rows
    for numel, dt in SWEEP:
        if max_numel is not None and numel > max_numel:
            continue
        watchdog.enter("dist round sweep %d %s" % (numel, dt), 900.0)
        dtype = torch.float32 if dt == "f32" else torch.bfloat16
        esize = 4 if dt == "f32" else 2
        # parameters, two snapshot slots, staging (two under the board), relay buffer + margin:
        # checked on every rank before anything is allocated, so no rank fails alone inside the
        # binding collectives
        if not vmm_ok and numel * esize >= VMM_MIN_BYTES:
            rows.append({"numel": numel, "dtype": dt, "transport": pull,
                         "error": "not run: its snapshot slots are fd-shared hipMemCreate chunks, and a +vmm parity "
                                  "transport failed on these devices"})
            progress("dist sweep %d %s skipped: %s" % (numel, dt, rows[-1]["error"]))
            continue
        need = 6 * numel * esize + (2 << 30)
        free = torch.cuda.mem_get_info(device)[0]
        if not _agree(free >= need * share, world, ctl):
            rows.append({"numel": numel, "dtype": dt, "transport": pull,
                         "error": "device memory: %.1f GB needed per rank, %.1f GB free on rank %d for %d rank(s)"
                                  % (need / 1e9, free / 1e9, rank, share)})
            progress("dist sweep %d %s skipped: %s" % (numel, dt, rows[-1]["error"]))
            continue
        conn, flat, err, el, averaged, steps = None, None, None, None, 0, 0
        try:
            flat = torch.empty(numel, dtype=dtype, device=device)
            flat.normal_(generator=torch.Generator(device=device).manual_seed(rank))
            conn = DpwaConnection(names[rank], cfg, seed=1000 + rank, group="async" if sel_async else "lockstep",
                                  pull=mode)
            if resident:
                conn.make_resident(flat)
                del flat
                flat = None

            def step():
                f = conn.parameters if resident else flat
                conn.update_send(f, 1.0, reuse_snapshot=write_through)
                return conn.update_wait_average(f, 1.0, write_through=write_through)[0] is not None

            for _ in range(warmup):
                step()
            torch.cuda.synchronize()
            dist.barrier(group=ctl)
            t0 = time.perf_counter()      # one more round sizes the timed run: >= ~0.25 s, 3..50 rounds
            step()
            torch.cuda.synchronize()
            got = [None] * world
            dist.all_gather_object(got, time.perf_counter() - t0, group=ctl)
            steps = int(min(50, max(min_steps, np.ceil(0.25 / max(got)))))
            dist.barrier(group=ctl)
            t0 = time.perf_counter()
            averaged = sum(step() for _ in range(steps))
            torch.cuda.synchronize()
            dist.barrier(group=ctl)
            el = time.perf_counter() - t0
        except Exception as e:   # noqa: BLE001 -- the size is reported failed, the sweep goes on
            err = "%s: %s" % (type(e).__name__, e)
            progress("dist sweep %d %s FAILED: %s" % (numel, dt, err))
        ok = _agree(err is None, world, ctl)
        got = [None] * world
        dist.all_gather_object(got, (el, averaged), group=ctl)
        if ok:
            el_max = max(g[0] for g in got)
            av = sum(g[1] for g in got)
            rows.append({"numel": numel, "dtype": dt, "value": round(av * 3 * numel * esize / el_max / 1e9, 1),
                         "ms_per_step": round(1e3 * el_max / steps, 3),
                         "gossip_rounds_per_s": round(world * steps / el_max, 1), "averagings": int(av),
                         "steps": steps, "transport": pull,
                         "publish": "resident" if resident else "write-through" if write_through else "full"})
            progress("dist sweep %d %s: %.1f GB/s" % (numel, dt, rows[-1]["value"]))
        else:
            rows.append({"numel": numel, "dtype": dt, "error": err or "failed on another rank", "transport": pull})
        if conn is not None:
            try:
                conn.close()
            except Exception as e:   # noqa: BLE001
                progress("dist sweep close: %s" % e)
        del conn, flat
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        dist.barrier(group=ctl)
    return rows


def cold_rounds(device, cfg_dir, numel, dtype, steps, warmup=2, publish="write-through", min_bytes=1.2e9):
    """SURVEY §8(d) cache honesty for the whole round: the timed loop of the N=1 line over K
    self-peer learners taken in turn (round i runs learner i mod K), K chosen so more than
    `min_bytes` of other learners' buffers are touched between two rounds of one learner -- the
    256 MiB Infinity Cache holds nothing a round re-reads.  Same calls as the timed loop
    (update_send with the write-through snapshot, update_wait_average); value = 3*N*s per
    completed averaging over the wall time."""
    from dpwa_amd import DpwaConnection
    from dpwa_amd.group import LocalGroup
    esize = 4 if dtype == torch.float32 else 2
    per = 3 * numel * esize         # what one round touches: parameters, published slot, next slot
    # (at most 32 learners -- a stream and events each; small vectors then rotate less than
    # min_bytes, and bytes_between_reuses says how much)
    K = 1 if per >= min_bytes else min(32, max(2, int(np.ceil(min_bytes / per)) + 1))
    wt = publish == "write-through"
    conns, flats = [], []
    for k in range(K):
        cfg = os.path.join(cfg_dir, "cold_%d.yaml" % k)
        write_config(cfg, ["c%d" % k], "constant", self_peer=True, base_port=45600 + k)
        conns.append(DpwaConnection("c%d" % k, cfg, seed=2000 + k, group=LocalGroup()))
        f = torch.empty(numel, dtype=dtype, device=device)
        f.normal_(generator=torch.Generator(device=device).manual_seed(k))
        flats.append(f)

    def step(i):
        c, f = conns[i % K], flats[i % K]
        c.update_send(f, 1.0, reuse_snapshot=wt)
        return c.update_wait_average(f, 1.0, write_through=wt)[0] is not None

    for i in range(warmup * K):
        step(i)
    n = max(steps, 20 * K)          # every learner set at least 20 times
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    averaged = sum(step(i) for i in range(n))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for c in conns:
        c.close()
    del conns, flats
    torch.cuda.empty_cache()
    return {"value": round(averaged * 3 * numel * esize / el / 1e9, 2), "ms_per_step": round(1e3 * el / n, 4),
            "gossip_rounds_per_s": round(n / el, 1), "steps": n, "learner_sets": K,
            "bytes_between_reuses": (K - 1) * per, "publish": publish,
            "basis": "the timed loop's rounds over %d self-peer learners in turn: %.2f GB of other learners' "
                     "buffers between two rounds of one learner (Infinity Cache 256 MiB), so every round reads "
                     "HBM" % (K, (K - 1) * per / 1e9)}


def adapter_loop(device, cfg_dir, numel, dtype, steps, warmup=5):
    """The drop-in itself: DpwaPyTorchAdapter (pytorch.py:37-68's API) over a model holding one
    parameter of `numel` elements, configs[1]'s self-peer YAML, the adapter's defaults
    (write-through, reuse guard on) -- update_send, update_wait per round, no training step -- and
    the same with reuse_guard=False.  What the connection-level line costs through the adapter:
    its host work per call and, with the guard, the two small kernels per update_send that check
    sampled words of the parameters against the snapshot the average wrote.  Also the
    resident adapter (resident=True) with and without its window guard (the reuse_guard flag there:
    sampled words saved at update_send, compared at update_wait), the learner its own peer
    as in the line."""
    from dpwa_amd import DpwaPyTorchAdapter
    from dpwa_amd.group import LocalGroup
    esize = 4 if dtype == torch.float32 else 2
    out = {}
    for i, (key, guard, resident) in enumerate((("default", True, False), ("no_guard", False, False),
                                                 ("resident", True, True), ("resident_no_guard", False, True))):
        cfg = os.path.join(cfg_dir, "adapter_%s.yaml" % key)
        write_config(cfg, ["a1"], "constant", self_peer=True, base_port=45400 + 2 * i)
        net = torch.nn.Module()
        g = torch.Generator(device=device).manual_seed(0)
        net.register_parameter("w", torch.nn.Parameter(torch.randn(numel, device=device, generator=g).to(dtype)))
        ad = DpwaPyTorchAdapter(net, "a1", cfg, seed=3000, group=LocalGroup(), reuse_guard=guard, resident=resident)
        for _ in range(warmup):
            ad.update_send(1.0)
            ad.update_wait(1.0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            ad.update_send(1.0)
            ad.update_wait(1.0)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[key] = {"value": round(steps * 3 * numel * esize / el / 1e9, 2), "ms_per_step": round(1e3 * el / steps, 4),
                    "reuse_guard": guard, "resident": resident,
                    "guard_hits": ad.window_guard_hits if resident else ad.reuse_guard_hits}
        ad.connection.close()
        del ad, net
        torch.cuda.empty_cache()
    out["note"] = ("DpwaPyTorchAdapter(net, name, config) over one %d-element parameter, self-peer config, "
                   "update_send -> update_wait, %d steps; value = 3*N*s per averaging / wall time. The resident "
                   "rows' learner reads its parameters and its peer from the same slot (it is its own peer), so "
                   "their kernel moves 2*N*s and their value is no HBM rate" % (numel, steps))
    return out


def co_resident_pair(device, cfg_dir, numel, dtype, steps, warmup=5, cold=True):
    """Round 4's N=1 line, kept as an extra: two resident learners co-resident on one GPU that
    average with each other (each the other's only peer), both averages in one dispatch
    (k_lerp_pair: one workgroup per span loads both published slots once and stores both
    averages).  Two averagings (2 x 3*N*s of the metric's unit) move 4*N*s through HBM, so the
    metric-unit rate exceeds what HBM moves; `hbm` prices the dispatch on the bytes it moves."""
    from dpwa_amd import DpwaConnection
    from dpwa_amd.group import LocalGroup
    esize = 4 if dtype == torch.float32 else 2
    cfg = os.path.join(cfg_dir, "pair.yaml")
    write_config(cfg, ["w1", "w2"], "constant", base_port=45500)
    group = LocalGroup()
    conns = []
    for g, nm in enumerate(("w1", "w2")):
        c = DpwaConnection(nm, cfg, seed=1000 + g, group=group)
        f = torch.empty(numel, dtype=dtype, device=device)
        f.normal_(generator=torch.Generator(device=device).manual_seed(g))
        c.make_resident(f)
        del f
        conns.append(c)

    def step():
        for c in conns:
            c.update_send(c.parameters, 1.0)
        res = DpwaConnection.update_wait_average_many(conns, [c.parameters for c in conns], [1.0, 1.0])
        return sum(p is not None for p, _ in res)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    averaged = sum(step() for _ in range(steps))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for c in conns:
        c.close()
    del conns
    torch.cuda.empty_cache()
    out = {"value": round(averaged * 3 * numel * esize / el / 1e9, 2), "ms_per_step": round(1e3 * el / steps, 4),
           "gossip_rounds_per_s": round(averaged / el, 1), "steps": steps, "learners": 2,
           "kernel": "dpwa::k_lerp_pair (two resident learners averaging with each other in one dispatch)",
           "value_note": "3*N*s per averaging, two averagings per round; they share their two snapshot reads, "
                         "so this is not an HBM rate (it can exceed the HBM peak)"}
    if cold:
        c = cold_kernel(numel, dtype, device, False, learners=2, resident=True, pair=True)
        hb = 4 * numel * esize
        out["hbm"] = {"bytes_per_launch": hb, "avg_launch_us": round(c["avg_launch_us"], 2),
                      "achieved": round(hb / (c["avg_launch_us"] * 1e-6) / 1e9, 1),
                      "frac": round(hb / (c["avg_launch_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                      "basis": "cold (rotating buffers), the 4*N*s the dispatch moves"}
        out["algorithmic_gbs"] = round(6 * numel * esize / (c["avg_launch_us"] * 1e-6) / 1e9, 1)
    return out


def size_sweep(device, rows=None):
    """The averaging kernel, cold, per launch, at every north_star size (11.17M/100M fp32,
    1B/7B bf16), in every publish form: plain (3*N*s bytes per launch), write-through
    (4*N*s: the next snapshot is written by the same pass) and resident (3*N*s: read one slot,
    write the other); and at 11.17M / 100M the batched dispatch of two learners' averages (the
    N=1 loop's kernel, 2 x the form's bytes)."""
    rows = [] if rows is None else rows
    for numel, dt in SWEEP:
        esize = 4 if dt == "f32" else 2
        forms = [("full", 1), ("write-through", 1), ("resident", 1)]
        if numel <= 100_000_000:
            forms += [("write-through", 2), ("resident", 2)]
        for form, learners in forms:
            wt = form == "write-through"
            pair = form == "resident" and learners == 2      # the N=1 loop's mutual pair (4*N*s)
            c = cold_kernel(numel, torch.float32 if dt == "f32" else torch.bfloat16, device, wt, learners=learners,
                            resident=form == "resident", pair=pair)
            nbytes = 4 * numel * esize if pair else learners * (4 if wt else 3) * numel * esize
            gbs = nbytes / (c["avg_launch_us"] * 1e-6) / 1e9
            rows.append({"numel": numel, "dtype": dt, "publish": form,
                         "learners_per_launch": learners, "mutual_pair": pair,
                         "bytes_per_launch": nbytes, "avg_launch_us": round(c["avg_launch_us"], 2),
                         "median_launch_us": round(c["median_launch_us"], 2), "achieved": round(gbs, 1),
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "launches": c["launches"],
                         "rotating_buffer_sets": c["rotating_buffer_sets"],
                         "batch_bracket_us": round(c["batch_bracket_us"], 2)})
    return rows


SCALING_DEFINITION = ("one learner per GPU at every N (N=1: its peer is its own snapshot, configs[1]; N>1: one "
                      "rank per GPU, peers over xGMI), the same publish form at every N.  raw = aggregate "
                      "gossip rounds/s of the bandwidth loop (update_send -> update_wait, no training step): "
                      "HBM-bound at N=1, xGMI-bound at N>1, so its N-ratio cannot reach 6x (DESIGN §6).  "
                      "weak = aggregate rounds/s with a fixed synthetic training step per learner (bf16 GEMMs "
                      "+ a write of every parameter) between update_send and update_wait, the reference's loop "
                      "(main.py:130-145, SURVEY §7/§8d C4): per-learner work is fixed, so its N-ratio is the "
                      "weak-scaling figure")


def scaling_basis(world, learners_per_gpu, publish, rounds, elapsed, value, overlap):
    """The line's `scaling_basis`: the same keys at every N (tests/test_bench_host.py checks it), so
    the driver's 1/2/4/8-GPU lines compare like with like."""
    learners = world * learners_per_gpu
    raw = rounds / elapsed if elapsed else None
    weak = {"gossip_rounds_per_s": None, "gossip_rounds_per_s_per_learner": None, "ms_per_step": None,
            "compute_only_ms_per_step": None, "gossip_overhead_frac": None}
    if overlap is not None:
        weak.update(gossip_rounds_per_s=overlap["gossip_rounds_per_s"],
                    gossip_rounds_per_s_per_learner=round(overlap["gossip_rounds_per_s"] / learners, 1),
                    ms_per_step=overlap["ms_per_step"], compute_only_ms_per_step=overlap["compute_only_ms_per_step"],
                    gossip_overhead_frac=overlap["gossip_overhead_frac"])
    return {"definition": SCALING_DEFINITION, "n_gpus": world, "learners_per_gpu": learners_per_gpu,
            "learners": learners, "publish": publish,
            "raw": {"gossip_rounds_per_s": round(raw, 1) if raw else None,
                    "gossip_rounds_per_s_per_learner": round(raw / learners, 1) if raw else None,
                    "value": value, "loop": "update_send -> update_wait (no training step)"},
            "weak": dict(weak, loop="update_send -> step (GEMMs, then a write of every parameter) -> update_wait")}


# ---------------------------------------------------------------- the run
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if args.gpus > 1 and world == 0:
        # no launcher: start one as a child process before anything touches a GPU
        sys.exit(self_launch(args, argv))
    world = world or 1
    # stdout carries exactly one line: keep a dup of it for emit() and send everything else that
    # writes to fd 1 (print, C++ libraries) to stderr
    global _RESULT_FD
    sys.stdout.flush()
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)
    # a rank stopped from outside (the launcher after another rank failed, a time limit) prints
    # where every thread was before it goes
    import faulthandler
    import signal
    faulthandler.register(signal.SIGTERM, all_threads=True, chain=True)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    if world == 1 and args.publish == "resident":
        raise SystemExit("--publish resident at N=1: the line's learner averages with its own snapshot "
                         "(configs[1]'s self-peer), which resident parameters would read twice from one slot; "
                         "the resident co-resident pair is the line's `co_resident_pair` block")
    global _WATCHDOG
    wd = _WATCHDOG = Watchdog(args, world, rank)
    # the CPU baseline first, before anything touches the GPU (its learners are child processes)
    wd.enter("start: world %d, numel %d %s" % (world, args.numel, args.dtype), 600.0)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        wd.enter("cpu baseline", 600.0 + 20.0 * args.cpu_seconds)
        cpu = cpu_baseline(args.numel, args.cpu_seconds, rows=not args.no_cpu_rows)
    # one GPU per rank; the modulo only matters for rehearsals with more ranks than GPUs
    wd.enter("gpu init", 600.0)
    device = torch.device("cuda", local_rank % torch.cuda.device_count())
    torch.cuda.set_device(device)
    ctl = None
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:   # rehearsal of the N>1 path on fewer GPUs (RCCL refuses two ranks per GPU)
            dist.init_process_group("gloo")
        ctl = dist.new_group(backend="gloo")    # control plane: object gathers, agreement, host barriers

    def hbarrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier(group=ctl)

    from dpwa_amd import DpwaConnection
    from dpwa_amd import _lib
    from dpwa_amd.group import LocalGroup

    dtype = torch.float32 if args.dtype == "f32" else torch.bfloat16
    esize = 4 if dtype == torch.float32 else 2
    tmp = tempfile.mkdtemp(prefix="dpwa_bench_")
    cfg = os.path.join(tmp, "bench.yaml")
    if world == 1:
        # configs[1]: one learner whose peer is its own snapshot (a node entry at its own address)
        names = ["w1"]
        write_config(cfg, names, args.interpolation, args.fetch_probability, args.divergence_threshold,
                     self_peer=True)
        mine = [(names[0], 0)]
    else:
        names = ["w%d" % (r + 1) for r in range(world)]
        write_config(cfg, names, args.interpolation, args.fetch_probability, args.divergence_threshold)
        mine = [(names[rank], rank)]

    # The parity leg runs first: at N>1 a transport that fails it on this node's devices is
    # reported (parity: false) and left out of the trials, so the timed run always uses a
    # transport whose results matched the oracle; at N=1 it checks both local forms (and gives
    # the GPU a second of work between the CPU baseline and the timed rounds).  At N>1 the
    # fd-shared (+vmm) forms are checked after the line is held (late_parity): no timed transport
    # uses them (they only gate the sweep's sizes above VMM_MIN_BYTES), so a hang in an import
    # path the line does not depend on costs the watchdog's phase, not the measured line.
    # Before the others, at N>1, lockstep/copy alone: once it passed, a provisional line is
    # measured on it and held (provisional_line), so the driver's multi-GPU run keeps a verified
    # measurement whatever the less plain transports do on its devices.
    parity = None
    late_parity = []
    if not args.no_parity:
        transports = parity_transports(world, args.gossip)
        late_parity = [t for t in transports if "+vmm" in t] if world > 1 else []
        early = [t for t in transports if t not in late_parity]
        first = early[:1] if world > 1 and early[:1] == ["lockstep/copy"] else []
        parity = parity_leg(world, rank, local_rank, device, tmp, first, args.dist_backend, ctl=ctl,
                            watchdog=wd) if first else {}
        if first and parity.get("lockstep/copy") and not args.no_provisional:
            ok, prov = provisional_line(args, world, rank, device, cfg, mine, dtype, ctl, wd, parity)
            if ok:
                wd.hold(prov, 0)
        parity.update(parity_leg(world, rank, local_rank, device, tmp, early[len(first):], args.dist_backend,
                                 ctl=ctl, watchdog=wd))

    # rehearsals run several ranks on one GPU: their pulls never cross an xGMI link
    shared_device = world > 1 and world > torch.cuda.device_count()
    wd.enter("learners", 300.0)
    group = LocalGroup() if world == 1 else None
    learners = []
    for name, seed in mine:
        g = torch.Generator(device=device).manual_seed(seed)
        flat = torch.randn(args.numel, device=device, generator=g, dtype=torch.float32).to(dtype)
        # under a DistGroup the relay buffers are allocated up front so every transport can be tried
        conn = DpwaConnection(name, cfg, seed=1000 + seed, group=group if world == 1 else "lockstep",
                              pull="relay" if world > 1 else None)
        learners.append((conn, flat))
    resident_main = args.publish == "resident"
    publish_fallback = None
    if resident_main and parity is not None:
        # the timed run must use a verified form: if no resident transport passed the parity check
        # but a write-through/full one did (the same on every rank: the verdicts are agreed), time
        # the write-through form instead and say so in the line
        res_ok = any(v for k, v in parity.items() if "+res" in k)
        other_ok = any(v for k, v in parity.items() if k != "workload" and "+res" not in k)
        if not res_ok and other_ok:
            resident_main = False
            args.publish = "write-through"
            publish_fallback = "no resident transport passed the parity check: write-through timed instead"
            progress(publish_fallback)
    if resident_main:
        # the parameters move into each learner's own snapshot slots (binds it: at N>1 every rank
        # runs this in the same order, the binding's exchange is collective)
        for conn, flat in learners:
            conn.make_resident(flat)

    stream = torch.cuda.current_stream(device)
    # co-resident learners on their own streams (their kernels overlap) or all on one
    streams = ([torch.cuda.Stream(device) for _ in learners] if args.streams == "per-learner"
               else [stream for _ in learners])
    batched = world == 1 and args.streams == "one" and not args.no_batch and len(learners) > 1
    # per-learner loss stream: constant 1.0, or SURVEY §8d C4's synthetic decay
    # l_t = 2 exp(-t/200) + 0.05 U(0,1) (seeded per learner) so a divergence threshold is crossed
    loss_rngs = [np.random.default_rng(7 + seed) for _, seed in mine]
    loss_t = [0]

    def loss_of(i):
        if args.loss_schedule == "constant":
            return 1.0
        return 2.0 * float(np.exp(-loss_t[0] / 200.0)) + 0.05 * float(loss_rngs[i].random())

    def run(steps, warmup, write_through, sample_every=0, warmup_s=0.0):
        """`steps` timed lock-step rounds.  sample_every == 0: nothing but the rounds (the
        pass `value` comes from).  sample_every = k > 0: the averaging dispatch of every k-th
        step is timed by its own dispatch events (and/or bracketed by an event pair on its
        stream) -- the in-loop kernel figure, from a separate pass.  warmup_s: after the
        `warmup` rounds, more untimed rounds up to about that many seconds in all (a count agreed
        by every rank from the warmup rounds' time)."""
        lerp_events = []
        sampled = []        # batched: per timed dispatch (learner whose pair timed it, averages in it)
        n_slots = (steps // sample_every + 1) * len(learners) if sample_every else 0
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(n_slots)]
        lib = _lib.load()
        timed_learners = []

        conns_ = [c for c, _ in learners]
        # resident learners: their parameters are where the learner keeps them (read once a round)
        resident = conns_[0]._learner is not None and conns_[0].parameters is not None
        flats_ = [c.parameters for c in conns_] if resident else [f for _, f in learners]
        one_stream = all(st is stream for st in streams)
        const_loss = [1.0] * len(learners) if args.loss_schedule == "constant" else None

        def step(k, timed):
            done = 0
            losses = const_loss or [loss_of(i) for i in range(len(learners))]
            loss_t[0] += 1
            for i, conn in enumerate(conns_):
                if one_stream:      # (a stream context costs microseconds of host time per round)
                    conn.update_send(flats_[i], losses[i], reuse_snapshot=write_through)
                else:
                    with torch.cuda.stream(streams[i]):
                        conn.update_send(flats_[i], losses[i], reuse_snapshot=write_through)
            sample = timed and sample_every and k % sample_every == 0
            if batched:
                if sample:
                    a, b = events[len(sampled)]
                    if args.timing != "dispatch":
                        a.record(stream)
                    if args.timing != "bracket":      # the dispatch takes its first armed learner's pair
                        for c in timed_learners:
                            lib.dpwa_learner_arm_timing(c._learner.handle)
                res = DpwaConnection.update_wait_average_many(conns_, flats_, losses, write_through=write_through)
                if resident:
                    flats_[:] = [c.parameters for c in conns_]
                got = [p is not None for p, _ in res]
                if sample and any(got):
                    sampled.append((got.index(True), sum(got)))     # (pair owner, averages in the dispatch)
                    if args.timing != "dispatch":
                        b.record(stream)
                        lerp_events.append((a, b))
                return sum(got)
            for i, conn in enumerate(conns_):
                flat = flats_[i]
                st = streams[i]
                with (_NoCtx if one_stream else torch.cuda.stream(st)):
                    # the adapter's update_wait: fused device factor + lerp (one kernel)
                    if sample:
                        a, b = events[len(lerp_events)]
                        if world > 1 and args.timing != "dispatch":   # keep the pull wait out of the bracket
                            lib.dpwa_learner_wait_fetch(conn._learner.handle, st.cuda_stream)
                        if args.timing != "dispatch":
                            a.record(st)
                        if args.timing != "bracket" and conn in timed_learners:
                            lib.dpwa_learner_arm_timing(conn._learner.handle)
                    payload, _ = conn.update_wait_average(flat, losses[i], write_through=write_through)
                    if resident:
                        flats_[i] = conn.parameters
                    if sample and args.timing != "dispatch":
                        b.record(st)
                        if payload is not None:
                            lerp_events.append((a, b))
                done += payload is not None
            return done

        t_w = time.perf_counter()
        for k in range(warmup):
            step(k, False)
        if warmup_s > 0:
            torch.cuda.synchronize()
            per = (time.perf_counter() - t_w) / max(1, warmup)
            extra = int(min(200_000, max(0, np.ceil(warmup_s / max(per, 1e-6)) - warmup)))
            if world > 1:
                got = [None] * world
                dist.all_gather_object(got, extra, group=ctl)
                extra = max(got)
            for k in range(extra):
                step(k, False)
            warm_extra[0] = extra
        if sample_every:
            for conn, _ in learners:    # kernel-dispatch timing of the sampled averaging launches
                if conn._learner is not None:
                    _lib.call("dpwa_learner_time_averages", conn._learner.handle, steps // sample_every + 1)
                    timed_learners.append(conn)
        hbarrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        averaged = 0
        for k in range(steps):
            averaged += step(k, True)
        torch.cuda.synchronize()
        if world > 1:
            hbarrier()
        elapsed = time.perf_counter() - t0
        bracket_ms = np.array([a.elapsed_time(b) for a, b in lerp_events]) if lerp_events else np.array([np.nan])
        kern_us, per_learner = [], []
        for conn in timed_learners:
            buf = (ctypes.c_float * max(1, len(events)))()
            cnt = ctypes.c_int()
            _lib.call("dpwa_learner_read_average_times", conn._learner.handle, buf, len(events), ctypes.byref(cnt))
            per_learner.append(list(buf[:cnt.value]))
            kern_us += list(buf[:cnt.value])
            _lib.call("dpwa_learner_time_averages", conn._learner.handle, 0)
        n_avg = np.ones(len(kern_us))       # averages per timed dispatch
        if batched and sampled and args.timing != "bracket":
            # each timed dispatch from its pair owner's list, in the order the dispatches ran
            kern_us, n_avg = [], []
            nxt = [0] * len(per_learner)
            for owner, n in sampled:
                if nxt[owner] < len(per_learner[owner]):
                    kern_us.append(per_learner[owner][nxt[owner]])
                    n_avg.append(n)
                    nxt[owner] += 1
            n_avg = np.array(n_avg, dtype=float)
        if args.timing == "bracket":
            kern_us = list(bracket_ms * 1e3)
            n_avg = np.array([n for _, n in sampled], dtype=float) if batched else np.ones(len(kern_us))
        lerp_ms = (np.array(kern_us) / 1e3 if kern_us else np.array([np.nan]), bracket_ms,
                   n_avg if len(n_avg) else np.array([np.nan]))
        stats = torch.tensor([elapsed, float(averaged), float(len(learners) * steps)], dtype=torch.float64)
        if world > 1:
            got = [None] * world
            dist.all_gather_object(got, stats.tolist(), group=ctl)
            return (max(g[0] for g in got), sum(g[1] for g in got), sum(g[2] for g in got), lerp_ms)
        return elapsed, float(averaged), float(len(learners) * steps), lerp_ms

    warm_extra = [0]      # untimed rounds the time-based warmup added to the main timed run

    def params_of(conn, flat):
        """Where a learner's parameters are now: its resident slot, else its flat buffer."""
        p = conn.parameters if conn._learner is not None else None
        return flat if p is None else p

    def make_compute(target_us):
        """A fixed-duration stand-in for a training step: k back-to-back
        4096^3 bf16 GEMMs on the compute stream, k calibrated to ~target_us."""
        a = torch.randn(4096, 4096, device=device, dtype=torch.bfloat16)
        b = torch.randn(4096, 4096, device=device, dtype=torch.bfloat16)
        c = torch.empty(4096, 4096, device=device, dtype=torch.bfloat16)
        for _ in range(5):
            torch.matmul(a, b, out=c)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            torch.matmul(a, b, out=c)
        e1.record()
        torch.cuda.synchronize()
        per_us = e0.elapsed_time(e1) * 1e3 / 20
        k = max(1, int(round(target_us / per_us)))
        if world > 1:            # every rank runs the same step
            got = [None] * world
            dist.all_gather_object(got, k, group=ctl)
            k = max(got)

        def compute():
            for _ in range(k):
                torch.matmul(a, b, out=c)
        return compute, k, per_us

    def run_overlap(steps, warmup, compute, gossip, wt, update):
        """The reference's training loop (main.py:130-145): update_send, the step (`compute`, then
        `update` -- an SGD-style write of every learner's parameters), update_wait.  The step
        writes the parameters while peers read the snapshot taken at update_send, so the learners
        are write-through (or full-publish) ones: a resident learner's update_wait refuses
        parameters written in that window."""
        def step():
            done = 0
            losses = [loss_of(i) for i in range(len(learners))]
            loss_t[0] += 1
            if gossip:
                for i, (conn, flat) in enumerate(learners):
                    conn.update_send(flat, losses[i], reuse_snapshot=wt)
            for _, flat in learners:
                compute()
                update(flat)
            if gossip:
                if batched:
                    res = DpwaConnection.update_wait_average_many([c for c, _ in learners],
                                                                  [f for _, f in learners], losses,
                                                                  write_through=wt)
                    done += sum(p is not None for p, _ in res)
                else:
                    for i, (conn, flat) in enumerate(learners):
                        payload, _ = conn.update_wait_average(flat, losses[i], write_through=wt)
                        done += payload is not None
            return done

        for _ in range(warmup):
            step()
        hbarrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            hbarrier()
        el = time.perf_counter() - t0
        if world > 1:
            got = [None] * world
            dist.all_gather_object(got, el, group=ctl)
            el = max(got)
        return el

    def set_pull(mode):
        for conn, _ in learners:
            conn.set_pull(mode)
        if world > 1:
            hbarrier()

    def verified(trial):
        return parity is None or parity.get(parity_key(trial), False)

    pull_trials = {}
    trial_errors = {}
    pull = args.pull
    wt_lockstep = args.publish == "write-through"     # lock-step rounds' publish form (resident: resident_main)
    res_sfx = "+res" if resident_main else ""
    lockstep_learners = list(learners)
    async_learners = []
    if world > 1:
        wd.enter("binding %d lock-step learner(s)" % len(learners), 600.0)
        run(2, 2, False)   # binds the learners (IPC exchange) before the transport is chosen
        modes = [args.pull] if args.pull != "auto" else ["copy", "kernel:256", "kernel:1024", "relay:32",
                                                         "relay:128", "relay:512", "relay-avg:32",
                                                         "relay-avg:128", "relay-avg:512"]
        cands = []          # (key, lockstep?, pull mode, write-through)
        if args.gossip != "async":
            cands += [(m + res_sfx, True, m, wt_lockstep) for m in modes if verified(m + res_sfx)]
        if args.gossip != "lockstep":
            wd.enter("binding free-running learner(s)", 600.0)
            # free-running rounds over the gossip board, same learners' initial parameters (a
            # second set of nodes: a connection's group is fixed at construction)
            for (name, seed), (_, flat) in zip(mine, lockstep_learners):
                conn = DpwaConnection(name, cfg, seed=1000 + seed, group="async", pull="copy")
                if resident_main:
                    conn.make_resident(flat)
                async_learners.append((conn, flat))
            learners[:] = async_learners
            run(2, 2, False)
            for m in [m for m in modes if not m.startswith("relay")]:
                for wt in ((True,) if wt_lockstep else (False,)):    # the line's publish form only
                    key = "async/" + m + ("+wt" if wt else res_sfx)
                    if verified(key):
                        cands.append((key, False, m, wt))
        # interleaved passes, each trial >= --trial-ms and >= 30 rounds; the median decides
        rounds_of = {key: 30 for key, _, _, _ in cands}
        for p in range(max(1, args.trial_passes)):
            for key, lock, m, wt in cands:
                if key in trial_errors:
                    continue
                wd.enter("trial %s (pass %d)" % (key, p + 1), 120.0)
                err = None
                try:
                    learners[:] = lockstep_learners if lock else async_learners
                    set_pull(m)
                    el, av, _, _ = run(rounds_of[key], 2, wt)
                    gbs = av * 3 * args.numel * esize / el / 1e9
                except Exception as e:   # noqa: BLE001 -- the transport leaves the trials
                    err, el, gbs = "%s: %s" % (type(e).__name__, e), None, None
                    progress("trial %s FAILED: %s" % (key, err))
                if not _agree(err is None, world, ctl):
                    trial_errors[key] = err or "failed on another rank"
                    continue
                pull_trials.setdefault(key, []).append(round(gbs, 2))
                if p == 0:   # same on every rank: el is the max over ranks
                    rounds_of[key] = max(30, int(np.ceil(args.trial_ms * 1e-3 / (el / rounds_of[key]))))
                progress("trial %s: %.1f GB/s" % (key, gbs))
        medians = {k: float(np.median(v)) for k, v in pull_trials.items()}
        if not medians:
            wd.idle()
            if rank == 0:
                out = dict(wd.held) if wd.held is not None else base_line(args, world)   # the provisional line
                out["error"] = "no transport passed the parity check and its trials"
                out["parity"] = parity
                out["trial_errors"] = trial_errors
                emit_final(out, detail_path(world))
            sys.exit(1)
        pull = max(medians, key=medians.get)
        if pull.startswith("async/"):
            learners[:] = async_learners
            set_pull(trial_mode(pull))
        else:
            learners[:] = lockstep_learners
            for conn, _ in async_learners:   # free their streams and slots (fewer HW queues in use)
                conn.close()
            async_learners = []
            hbarrier()
            set_pull(trial_mode(pull))
    # trial key: "<mode>[+res]" (lock-step, publish per --publish) or "async/<mode>[+wt|+res]"
    sel_async = pull.startswith("async/")
    sel_mode = trial_mode(pull)
    wt_main = pull.endswith("+wt") if sel_async else wt_lockstep
    form = "resident" if resident_main else "write-through" if wt_main else "full"
    wd.enter("timed run: %s, %s publish" % (pull, form), 600.0 + 0.05 * (args.steps + args.warmup))
    elapsed, averaged, rounds, _ = run(args.steps, args.warmup, wt_main, warmup_s=args.warmup_s)
    progress("timed run: %.4f ms/step" % (1e3 * elapsed / args.steps))
    # the averaging kernel inside the loop: a separate sampled pass of the same rounds
    wd.enter("in-loop kernel timing", 600.0)
    s_steps = max(args.steps, 8 * args.sample_every)
    s_el, _, _, (lerp_ms, bracket_ms, lerp_navg) = run(s_steps, 2, wt_main, args.sample_every)
    pull_us = []
    if world > 1 and not sel_mode.startswith("relay"):
        # the pull alone (side-stream events around each copying fetch), in a short extra run
        wd.enter("pull timing", 300.0)
        p_steps = max(20, args.steps // 4)
        for conn, _ in learners:
            _lib.call("dpwa_learner_time_fetches", conn._learner.handle, p_steps + 4)
        run(p_steps, 2, wt_main)
        for conn, _ in learners:
            buf = (ctypes.c_float * (p_steps + 4))()
            cnt = ctypes.c_int()
            _lib.call("dpwa_learner_read_fetch_times", conn._learner.handle, buf, p_steps + 4, ctypes.byref(cnt))
            pull_us += list(buf[2:cnt.value])     # the 2 warmup rounds' pulls are left out
            _lib.call("dpwa_learner_time_fetches", conn._learner.handle, 0)
        got = [None] * world
        dist.all_gather_object(got, float(np.mean(pull_us)) if pull_us else float("nan"), group=ctl)
        pull_us = [float(np.mean(got))]
    secondary = None
    main_set = list(learners)
    wt_set = None           # write-through learners: the reference loop's form (secondary, overlap)
    wt_key = None           # the parity transport that vouches for them
    if not resident_main:
        wt_set = main_set
    elif not args.no_secondary or args.compute_us > 0:
        # resident learners cannot leave their slots: the write-through form runs on a second set
        # of learners (same initial parameters, same transport; at N>1 every rank makes its own in
        # the same order, the binding is collective)
        wt_key = write_through_key(world, pull)
        if parity is None or parity.get(wt_key, False):
            wd.enter("write-through learners", 300.0)
            grp2 = LocalGroup() if world == 1 else ("async" if sel_async else "lockstep")
            wt_set = [(DpwaConnection(name, cfg, seed=1000 + seed, group=grp2, pull=None if world == 1 else sel_mode),
                       f0.clone()) for (name, seed), (_, f0) in zip(mine, main_set)]
        else:
            progress("write-through form not timed: %s did not pass the parity check" % wt_key)
    if not args.no_secondary and wt_set is not None:
        wd.enter("secondary publish form", 600.0)
        learners[:] = wt_set
        s_wt = True if resident_main else not wt_main    # the form the main run did not time
        s2 = run(args.steps, args.warmup, s_wt)
        s2_k = run(s_steps, 2, s_wt, args.sample_every)
        secondary = ("write-through" if s_wt else "full", s2, s2_k[3])
        learners[:] = main_set
    overlap = None
    if args.compute_us > 0 and wt_set is not None:
        wd.enter("overlap", 600.0)
        compute, k_gemm, gemm_us = make_compute(args.compute_us)
        upd = torch.randn(args.numel, device=device, dtype=torch.float32).mul_(1e-4).to(dtype)

        def update(flat):
            flat.sub_(upd)      # the optimizer's write of the parameters (3*N*s of HBM traffic)

        o_steps = max(20, args.steps // 4)
        o_wt = True if resident_main else wt_main
        progress("overlap: %d GEMMs per step, %s learners" % (k_gemm, "write-through" if o_wt else "full"))
        learners[:] = wt_set
        o_trials = {}
        o_mode = sel_mode
        modes_o = [o_mode]
        if world > 1 and o_mode != "copy" and args.pull == "auto":
            # the copy engine leaves every CU to the training step: try it beside the
            # pure-loop winner and keep the cheaper overlap
            modes_o = [m for m in (o_mode, "copy")
                       if verified(("async/" + m + ("+wt" if o_wt else "")) if sel_async else m)] or [o_mode]
        # interleaved pairs (step alone, step + gossip) per mode; the first pair is dropped (a run's
        # first phase meets different clocks) and the medians of the rest are compared
        t_c, t_b = [], {m: [] for m in modes_o}
        for _ in range(OVERLAP_PAIRS):
            t_c.append(run_overlap(o_steps, 3, compute, False, o_wt, update))
            for m in modes_o:
                if len(modes_o) > 1:
                    set_pull(m)
                t_b[m].append(run_overlap(o_steps, 3, compute, True, o_wt, update))
        t_compute = float(np.median(t_c[1:]))
        o_trials = {m: float(np.median(v[1:])) for m, v in t_b.items()}
        o_mode = min(o_trials, key=o_trials.get)
        t_both = o_trials[o_mode]
        if len(modes_o) > 1:
            set_pull(sel_mode)
        else:
            o_trials = {}
        learners[:] = main_set
        overlap = {
            "compute": "%d x bf16 GEMM 4096^3 per learner per step (%.1f us each)" % (k_gemm, gemm_us),
            "steps": o_steps,
            "pairs": "%d interleaved (step alone, step + gossip) pairs, the first dropped, medians" % OVERLAP_PAIRS,
            "compute_only_ms_per_step": round(1e3 * t_compute / o_steps, 4),
            "ms_per_step": round(1e3 * t_both / o_steps, 4),
            "gossip_overhead_frac": round(t_both / t_compute - 1.0, 4),
            "rounds_per_s_per_learner": round(o_steps / t_both, 1),
            "gossip_rounds_per_s": round(o_steps * len(wt_set) * world / t_both, 1),   # all learners, all ranks
            "transport": o_mode if world > 1 else "in-place HBM read of its own published snapshot (self-peer)",
            "publish": "write-through" if o_wt else "full",
            "loop_order": "update_send -> step (GEMMs, then a write of every parameter) -> update_wait",
            "note": "the reference's loop order (main.py:130-145; SURVEY §8d C4 weak scaling) with a synthetic "
                    "step that writes the parameters while peers read the update_send snapshot, so the learners "
                    "publish write-through (%s): the overhead the gossip round adds to a step of this length. "
                    "Scaling definition: per-learner compute is fixed, so gossip_rounds_per_s (all learners) "
                    "compared across N is the weak-scaling figure; value above is the raw bandwidth loop"
                    % ("a second set of learners: the timed run's are resident, which refuses this order"
                       if resident_main else "the timed run's learners"),
        }
        if o_trials:
            overlap["trials_ms_per_step"] = {m: round(1e3 * t / o_steps, 4) for m, t in o_trials.items()}
    if resident_main and wt_set is not None:
        hbarrier()      # every rank's pulls of these learners' slots are done
        for conn, _ in wt_set:
            conn.close()
        wt_set = None
    value_cold = None
    if world == 1 and not args.no_value_cold:
        # SURVEY §8(d) cache honesty for the whole round: the same loop over learner sets rotated
        # beyond the Infinity Cache
        wd.enter("value_cold", 600.0)
        value_cold = cold_rounds(device, tmp, args.numel, dtype, args.steps, publish=form)
    pair = None
    adapter = None
    if world == 1 and not args.no_secondary:
        wd.enter("adapter loop", 600.0)
        adapter = adapter_loop(device, tmp, args.numel, dtype, args.steps, warmup=args.warmup)
        wd.enter("co-resident pair", 600.0)
        pair = co_resident_pair(device, tmp, args.numel, dtype, args.steps, warmup=args.warmup, cold=not args.no_cold)

    if parity is not None:
        parity["workload"] = ("%d-element fp32 vector per learner, %d lock-step rounds (clock interpolation, "
                              "fetch_probability %g, seeded training-step deltas, write-through and split rounds "
                              "mixed; 'self': the N=1 line's form, one learner whose peer is its own snapshot, "
                              "write-through in the reference order; 'local': two learners, averages batched), "
                              "%d free-running rounds over the "
                              "gossip board; every learner's parameters, clocks and peers compared bit for bit with "
                              "oracle/gossip.py (lock-step) and oracle/async_check.py (per version read); '+vmm': "
                              "snapshot slots (and relay buffers) fd-shared hipMemCreate chunks, the configs[3]/[4] "
                              "path" % (PARITY_N, PARITY_T, PARITY_FP, PARITY_ASYNC_T))
    used = "self" if world == 1 else parity_key(pull)

    unit_bytes = 3 * args.numel * esize
    per_launch = len(learners) if batched else 1
    wt_kernel = wt_main and not resident_main      # resident: the kernel moves the averaging's 3*N*s only
    # the bytes the timed loop's averaging dispatch moves through HBM (PMC-confirmed, `traffic`):
    # write-through 4*N*s (read parameters, read the peer snapshot, write parameters, write the next
    # snapshot), full / resident 3*N*s
    kbytes = (4 if wt_kernel else 3) * args.numel * esize * per_launch
    # the same kernel alone, cold (rotating buffers, per-launch dispatch events): the roofline's basis
    cold = None
    forms_cold = {}         # every single-learner form at the workload size, cold
    mix = None
    if not args.no_cold:
        wd.enter("cold kernel", 300.0)
        # one learner: each timed launch interleaved with its access mix alone on the same buffers
        cold = cold_kernel(args.numel, dtype, device, wt_kernel, learners=per_launch, resident=resident_main,
                           mix=per_launch == 1)
        mix = cold.get("mix")
        for key, wt_, res_ in (("write_through", True, False), ("full", False, False), ("resident", False, True)):
            same = per_launch == 1 and res_ == resident_main and wt_ == wt_kernel
            c = cold if same else cold_kernel(args.numel, dtype, device, wt_, learners=1, resident=res_)
            b = (4 if wt_ else 3) * args.numel * esize
            forms_cold[key] = {"bytes_per_launch": b, "avg_launch_us": round(c["avg_launch_us"], 2),
                               "frac": round(b / (c["avg_launch_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
            tb, _ = pmc_traffic(None, "write-through" if wt_ else "resident" if res_ else "full", 1, args.numel,
                                args.dtype, "cold")
            if tb:
                forms_cold[key]["traffic_x"] = round(tb / b, 4)     # PMC HBM bytes / moved bytes
    wd.enter("report", 120.0)
    out = None
    if rank == 0:
        value = averaged * unit_bytes / elapsed / 1e9
        lerp_us = float(np.nanmean(lerp_ms) * 1e3)
        k1 = kbytes / per_launch
        live_gbs = float(np.nansum(lerp_navg * k1) / np.nansum(lerp_ms * 1e-3) / 1e9) if np.isfinite(lerp_us) \
            else float("nan")
        k_us = cold["avg_launch_us"] if cold else lerp_us
        achieved = kbytes / (k_us * 1e-6) / 1e9
        variant = form
        traffic, traffic_src = pmc_traffic(args.traffic, variant, per_launch, args.numel, args.dtype,
                                           "cold" if cold else "in-loop")
        ops = "Ops%s" % args.dtype.upper()
        if resident_main:
            kname = ("dpwa::k_lerp<%s, COEF_FUSED, true, 64, 8, true> (resident: fused device factor + lerp from "
                     "the published slot into the other)" % ops)
        else:
            kname = ("dpwa::k_lerp<%s, COEF_FUSED, %s> (fused device factor + lerp%s)"
                     % (ops, "true" if wt_main else "false", " + write-through of the next snapshot" if wt_main else ""))
        sb = scaling_basis(world, len(mine), form, rounds, elapsed, round(value, 2), overlap)
        out = base_line(args, world)
        out.update({
            "value": round(value, 2),
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "dtype": "f32" if dtype == torch.float32 else "bf16",
            "value_cold": value_cold,
            "scaling_basis": sb,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": kname,
                "bytes_per_launch": kbytes,
                "bytes_note": ("4*N*s moved per averaging: read parameters, read the peer snapshot, write "
                               "parameters, write the next snapshot (the publish then copies nothing)" if wt_kernel else
                               "3*N*s moved per averaging: read the parameters, read the peer snapshot, write the "
                               "result"),
                "metric_bytes_per_averaging": unit_bytes,
                "avg_launch_us": round(k_us, 2),
                "basis": ("cold: the kernel alone over rotating buffers (> 1.2 GB between reuses), every launch "
                          "timed by its dispatch begin/end events, mean of %d" % cold["launches"]) if cold else
                         "in-loop (--no-cold)",
                "traffic_source": traffic_src,
                "traffic_x": round(traffic / kbytes, 4) if traffic else None,
                "in_loop_frac": round(live_gbs / HBM_PEAK_GBS, 4) if np.isfinite(live_gbs) else None,
                "in_loop_avg_launch_us": round(lerp_us, 2) if np.isfinite(lerp_us) else None,
                "learners_per_launch": per_launch,
                "cold": ({k: (round(v, 2) if isinstance(v, float) else v) for k, v in cold.items()}
                         if cold else None),
                "in_loop": {
                    "achieved": round(live_gbs, 1),
                    "frac": round(live_gbs / HBM_PEAK_GBS, 4),
                    "avg_launch_us": round(lerp_us, 2),
                    "launches_timed": int(np.isfinite(lerp_ms).sum()),
                    "timing": ("kernel dispatch begin/end events (hipExtLaunchKernelGGL) on the averaging "
                               "kernel's own stream" if args.timing != "bracket" else
                               "HIP event pair recorded around the launch on its stream")
                              + ", every %d-th step of a separate %d-step pass (not the timed one)"
                              % (args.sample_every, s_steps),
                    "sampled_pass_ms_per_step": round(1e3 * s_el / s_steps, 4),
                    "event_bracket_us": (round(float(np.nanmean(bracket_ms) * 1e3), 2)
                                         if args.timing != "dispatch" else None),
                    "note": ("inside the loop the learner re-reads what its last average wrote (134 MB at "
                             "configs[1], inside the 256 MiB Infinity Cache), so this live figure is warmer "
                             "than the cold basis; value_cold is the whole loop without that reuse"
                             if world == 1 else
                             "the averaging kernel of the timed rounds: it reads the staged peer snapshot (copy / "
                             "kernel / relay pulls) or, under relay-avg, the peer's stripes over xGMI itself, so "
                             "there it is link-bound and its bytes are not all HBM bytes"),
                },
                "forms_cold": forms_cold or None,
                "vs_measured_ceiling": {"gbs": HBM_MEASURED_GBS, "frac": round(achieved / HBM_MEASURED_GBS, 4),
                                        "source": "MI355X_MICROARCH.md: 6.29 TB/s measured for a float4 copy "
                                                  "(79 % of the 8 TB/s spec); peak above stays the spec"},
            },
            "config": {
                "workload": ("%ssynthetic %d-element %s vector, %s, %s interpolation, fetch_probability %g, "
                             "divergence_threshold %g, %s loss, %s publish"
                             % ("configs[1]: " if args.numel == RESNET18_NUMEL and world == 1 else "", args.numel,
                                args.dtype, "one learner, its peer its own snapshot (self-peer)" if world == 1 else
                                "one learner per GPU, %s rounds" % ("free-running" if sel_async else "lock-step"),
                                args.interpolation, args.fetch_probability, args.divergence_threshold,
                                args.loss_schedule, variant)),
                "learners": int(rounds / args.steps),
                "learners_per_gpu": len(mine),
                "numel": args.numel,
                "publish": variant,
                "loop_order": ("update_send -> update_wait -> step" if resident_main else
                               "update_send -> step -> update_wait (README.md:18-29, main.py:130-145); the timed "
                               "rounds have no step, scaling_basis.weak has one"),
                "peer": ("its own published snapshot: a second YAML node entry at the learner's own host:port, "
                         "which the reference's TxThread dials like any peer (conn.py:246-251)" if world == 1 else
                         "a random other rank's snapshot (TxThread's choice), pulled over xGMI (%s)" % sel_mode),
                "value_cold": value_cold["value"] if value_cold else None,
                "frac_moved_bytes_cold": round(achieved / HBM_PEAK_GBS, 4),
                "scaling_raw_rounds_per_s": sb["raw"]["gossip_rounds_per_s"],
                "scaling_weak_rounds_per_s": sb["weak"]["gossip_rounds_per_s"],
                "adapter_loop_value": adapter["default"]["value"] if adapter else None,
                "co_resident_pair_value": pair["value"] if pair else None,
                "parallelism": "gossip x%d" % int(rounds / args.steps),
                "streams": args.streams,
            },
            "value_basis": "the timed pass carries no instrumentation (no kernel timing, no events); value = 3*N*s "
                           "per completed averaging (SURVEY 8d's unit) over the wall time",
            "gossip_rounds_per_s": round(rounds / elapsed, 1),
            "gossip_rounds_per_s_per_learner": round(rounds / elapsed / (rounds / args.steps), 1),
            "averagings": int(averaged),
            "warmup_rounds": {"steps": args.warmup, "time_based_extra": warm_extra[0], "warmup_s": args.warmup_s,
                              "note": "untimed rounds before the timed steps: W, then more up to about warmup_s "
                                      "seconds in all, so the timed steps run at steady-state clocks"},
        })
        if mix is not None:
            out["roofline"]["mix_ceiling_frac"] = mix["frac"]
            out["roofline"]["kernel_over_mix_ceiling"] = round(achieved / mix["achieved"], 4)
            out["roofline"]["mix_ceiling"] = dict(mix, note=(
                "the timed kernel's access mix alone (same loads and stores at the same addresses, same launch "
                "shape and cache policy, no factor or lerp), each launch interleaved with a product launch in the "
                "same cold rotation: what one launch of this size reaches on this chip (kernel_over_mix_ceiling "
                "= the product kernel's rate over it)"))
        if wt_kernel and args.numel == RESNET18_NUMEL and args.dtype == "f32":
            out["roofline"]["vs_mix_ceiling"] = dict(MIX_CEILING_11M, kernel_frac_over_ceiling=round(
                achieved / HBM_PEAK_GBS / MIX_CEILING_11M["frac"], 4),
                note="round 2's stream_tune ceiling for one 11.17M-element 2R:2W launch (mix_ceiling: this run's)")
        if adapter is not None:
            out["adapter_loop"] = adapter
        if pair is not None:
            out["co_resident_pair"] = pair
        if publish_fallback:
            out["publish_fallback"] = publish_fallback
        if pull_trials:
            out["pull_trials_gbs"] = pull_trials
            out["pull_trials_median_gbs"] = {k: round(float(np.median(v)), 2) for k, v in pull_trials.items()}
            out["pull_choice"] = {"chosen": pull, "rule": "highest median over %d interleaved passes, each trial >= "
                                  "%g ms and >= 30 rounds" % (args.trial_passes, args.trial_ms)}
        if trial_errors:
            out["trial_errors"] = trial_errors
        if world > 1:
            pull_bytes = 256 + args.numel * esize
            p_us = pull_us[0] if pull_us and np.isfinite(pull_us[0]) else None
            p_gbs = pull_bytes / (p_us * 1e-6) / 1e9 if p_us else None
            out["xgmi"] = {
                "bytes_per_pull": pull_bytes,
                "avg_pull_us": round(p_us, 2) if p_us else None,
                "achieved_gbs_per_pull": round(p_gbs, 1) if p_gbs else None,
                "peak_gbs": XGMI_LINK_DIR_GBS,
                "frac": round(p_gbs / XGMI_LINK_DIR_GBS, 4) if p_gbs and not shared_device else None,
                "ranks_share_device": shared_device,
                "note": "one pull = one peer snapshot, one direction of the direct link between the two GPUs, timed "
                        "by side-stream events around each copying fetch (mean over ranks; null for the relay); peak "
                        "= MI355X xGMI spec per link and direction (%.1f GB/s both ways)%s"
                        % (XGMI_LINK_GBS, "; ranks share a device here (a rehearsal): the pulls never cross a link, "
                           "so the rate is an HBM copy rate and frac is null" if shared_device else ""),
            }
            if sel_mode.startswith("relay"):
                # every directed link carries at most one stripe per phase, two per round
                link_bytes = 2 * ((args.numel * esize + 15) // 16 * 16) // world
                l_gbs = link_bytes / (elapsed / args.steps) / 1e9
                out["xgmi"]["relay"] = {
                    "bytes_per_link_per_round": link_bytes,
                    "round_us": round(1e6 * elapsed / args.steps, 2),
                    "achieved_gbs_per_link_direction": round(l_gbs, 1),
                    "peak_gbs": XGMI_LINK_DIR_GBS,
                    "frac": round(l_gbs / XGMI_LINK_DIR_GBS, 4) if not shared_device else None,
                    "note": "the relay's busiest directed link per round over the whole round's time "
                            "(barriers and the average included): a lower bound on the link rate",
                }
        if secondary is not None:
            s_form, (w_el, w_avg, w_rounds, _), (w_ms, _, w_n) = secondary
            s_wt = s_form == "write-through"
            w_us = float(np.nanmean(w_ms) * 1e3)
            w_bytes = (4 if s_wt else 3) * args.numel * esize * float(np.nanmean(w_n))
            out["secondary_publish"] = {
                "publish": s_form,
                "value": round(w_avg * unit_bytes / w_el / 1e9, 2),
                "ms_per_step": round(1e3 * w_el / args.steps, 4),
                "avg_launch_us": round(w_us, 2),
                "kernel_gbs": round(w_bytes / (w_us * 1e-6) / 1e9, 1),
                "note": "the same rounds with the other publish form (value from an uninstrumented pass, the kernel "
                        "from a sampled one). full: every publish copies the 2*N*s snapshot, then the 3*N*s "
                        "average; write-through: the averaging kernel also writes the next snapshot (4*N*s) and "
                        "the publish moves nothing",
            }
        if overlap is not None:
            out["overlap"] = overlap
        out["cpu_baseline"] = cpu
        if parity is not None:
            out["parity"] = parity
            out["parity_of_timed_transport"] = {"transport": used, "ok": bool(parity.get(used, False))}
            out["parity_failed"] = sorted(k for k, v in parity.items() if k != "workload" and not v)
    # The sweeps over the north_star sizes come last: their rows go into the line as they are
    # measured, and a watchdog overrun in them prints the line built above (with the rows so
    # far and the error) and exits as the run would have.  Exit status: 1 when the timed
    # transport itself failed its parity check; a failure of any other transport (left out of
    # the trials, so never timed) is reported in the line's `parity` and on stderr, status 0, so
    # the measured, verified line is not discarded with it.
    parity_failed = parity is not None and not parity.get(used, False)
    size_rows, round_rows = [], []
    if out is not None and not args.no_sweep:
        if world == 1:
            out["roofline"]["size_sweep"] = size_rows
        out["round_sweep"] = round_rows
    code = 1 if parity_failed else 0
    wd.hold(out, code)
    # Everything after this point runs with the measurement done: an exception in it (a rank that
    # left a collective, a sweep size that does not fit) ends the job with the measured line
    # and the run's status, as a watchdog overrun does, never with a traceback in its place.
    printed = False
    try:
        if world == 1 and not args.no_sweep:
            wd.enter("size sweep", 900.0)
            size_sweep(device, rows=size_rows)
            wd.enter("round sweep", 900.0)
            round_sweep(device, tmp, rows=round_rows, publish=form)
        elif world > 1 and (late_parity or not args.no_sweep):
            # the timed learners' buffers go first: the sweep's 7B learner needs ~80 GB per GPU, and
            # the late parity transports build groups of their own
            for conn, _ in lockstep_learners + async_learners:
                conn.close()
            lockstep_learners, async_learners = [], []
            learners[:] = []
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            if late_parity:
                hbarrier()
                parity.update(parity_leg(world, rank, local_rank, device, tmp, late_parity, args.dist_backend, ctl=ctl,
                                         watchdog=wd))
                if out is not None:
                    out["parity_failed"] = sorted(k for k, v in parity.items() if k != "workload" and not v)
            if not args.no_sweep:
                vmm_ok = parity is None or all(v for k, v in parity.items() if "+vmm" in k)
                dist_round_sweep(world, rank, device, tmp, pull, wt_main, ctl, wd, max_numel=args.dist_sweep_max_numel,
                                 rows=round_rows, resident=resident_main, vmm_ok=vmm_ok)
        wd.enter("result", 60.0)
        if out is not None:
            emit_final(out, detail_path(world))
        printed = True
        wd.hold(None, code)      # the line is out: an overrun from here only exits
        wd.enter("shutdown", 300.0)
        for conn, _ in lockstep_learners + async_learners:
            conn.close()
        if world > 1:
            hbarrier()
            dist.destroy_process_group()
    except Exception as e:   # noqa: BLE001
        import traceback
        traceback.print_exc()
        progress("after the measured line, phase '%s': %s: %s" % (wd.phase, type(e).__name__, e))
        if not wd.disarm():      # the watchdog fired first: it prints the line and exits
            time.sleep(600)
        if out is not None and not printed:
            out["error"] = "after the measurement, phase '%s': %s: %s" % (wd.phase, type(e).__name__, e)
            out["phase"] = wd.phase
            if wd.transport is not None and isinstance(out.get("parity"), dict):   # a late parity check
                out["parity"][wd.transport] = False
                out["parity_failed"] = sorted(k for k, v in out["parity"].items() if k != "workload" and not v)
            emit_final(out, detail_path(world))
        sys.stderr.flush()
        os._exit(code)
    wd.idle()
    progress("done")
    if parity is not None:
        failed = sorted(k for k, v in parity.items() if k != "workload" and not v)
        if failed:
            print("bench.py: parity check FAILED for %s (timed transport %s: %s)"
                  % (failed, used, "ok" if not parity_failed else "FAILED"), file=sys.stderr, flush=True)
        if parity_failed:
            sys.exit(1)


if __name__ == "__main__":
    try:
        main()
    except Exception as e:   # noqa: BLE001 -- a held line (provisional or final) still goes out
        wd = _WATCHDOG
        if wd is None or wd.held_rc is None:
            raise
        if not wd.disarm():      # the watchdog fired first: it prints the line and exits
            time.sleep(600)
        import traceback
        traceback.print_exc()
        if wd.held is not None:
            out = dict(wd.held)
            out["error"] = "phase '%s': %s: %s (the held line)" % (wd.phase, type(e).__name__, e)
            out["phase"] = wd.phase
            if wd.transport is not None and isinstance(out.get("parity"), dict):
                out["parity"] = dict(out["parity"], **{wd.transport: False})
            emit_final(out, detail_path(wd.world))
        sys.stderr.flush()
        os._exit(wd.held_rc)     # as the watchdog would have exited
