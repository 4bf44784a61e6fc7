"""Node-list generation and launch helpers.

The reference's examples/pytorch-cifar/prepare.py:17-40 writes one localhost node per CPU core
into dpwa.yaml (from dpwa.yaml.t) and a run.sh with one ``taskset -c <core> python3 main.py
--name w<core> ...  &`` line per core.  On MI355X a node is a learner on a GPU, so ``prepare``
writes one node per GPU -- the reference's schema plus a per-node ``gpu:`` key, which the
reference's parser ignores (dpwa.py:66-72 makes each node a Struct) -- and a run.sh that
starts the job with torchrun, one rank per GPU; rank r is node r of the list and the trainer
finds its name and device with :func:`node_for_rank`.

  python -m dpwa_amd.launch prepare --gpus 8 --out-dir run/ --script main.py -- --lr=0.01 --batch-size 8
  python -m dpwa_amd.launch make-config --nodes 8 --out dpwa.yaml --interpolation clock --gpus 8
"""
import argparse
import os
import shlex
import stat
import sys

# dpwa.yaml.t (examples/pytorch-cifar/dpwa.yaml.t:1-23), same keys, same order
_TEMPLATE = """---
- nodes:
{nodes}

# The probability of initiating a fetch parameters request
- fetch_probability: {fetch_probability!r}

# The timeout value is used for flow-control
- timeout_ms: {timeout_ms}

# Choose interpolation method: clock, loss or constant
- interpolation: {interpolation}

# Diverge models when loss is reaching the value specified here (use 0 to disable)
- divergence_threshold: {divergence_threshold!r}

# Individual interpolation methods configuration:

- constant: {{ value: {constant_value!r} }}

- clock: 0

- loss: 0
"""


def config_text(names, fetch_probability=1, timeout_ms=2500, interpolation="constant", divergence_threshold=0.0,
                constant_value=0.5, host="localhost", base_port=45000, gpus=None, seed=None):
    """The reference schema (a list of single-key maps, dpwa/dpwa.py:29-51) for `names`.
    gpus: None, or one device index per node (the optional per-node `gpu:` key)."""
    if interpolation not in ("constant", "clock", "loss"):
        raise ValueError("interpolation must be constant, clock or loss")
    if gpus is not None and len(gpus) != len(names):
        raise ValueError("one gpu index per node")
    nodes = []
    for i, n in enumerate(names):
        extra = "" if gpus is None else ", gpu: %d" % gpus[i]
        nodes.append("  - {name: %s, host: %s, port: %d%s}" % (n, host, base_port + i, extra))
    text = _TEMPLATE.format(nodes="\n".join(nodes), fetch_probability=fetch_probability, timeout_ms=timeout_ms,
                            interpolation=interpolation, divergence_threshold=divergence_threshold,
                            constant_value=constant_value)
    if seed is not None:
        text += "\n- seed: %d\n" % seed
    return text


def write_config(path, names, fetch_probability=1, timeout_ms=2500, interpolation="constant",
                 divergence_threshold=0.0, constant_value=0.5, host="localhost", base_port=45000, seed=None,
                 gpus=None):
    """Writes config_text(...) to `path` and returns the path."""
    text = config_text(names, fetch_probability, timeout_ms, interpolation, divergence_threshold, constant_value,
                       host, base_port, gpus, seed)
    with open(path, "w") as f:
        f.write(text)
    return path


def node_for_rank(config_file, rank=None):
    """(node name, torch.device) of torch.distributed rank `rank` (default: $RANK): node r of
    the YAML list, on its `gpu:` (else $LOCAL_RANK, else r)."""
    import torch

    from .dpwa import DpwaConfiguration
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    cfg = DpwaConfiguration(config_file)
    nodes = cfg.get_nodes()
    if not 0 <= rank < len(nodes):
        raise ValueError("rank %d but the config lists %d nodes" % (rank, len(nodes)))
    name = nodes[rank]["name"]
    gpu = cfg.get_gpu(name)
    if gpu is None:
        gpu = int(os.environ.get("LOCAL_RANK", rank))
    return name, torch.device("cuda", gpu)


def run_script_text(n_ranks, script, script_args, config_file, master_port=29500):
    """run.sh (examples/pytorch-cifar/run.sh.t): the reference starts one background process
    per core and waits; here torchrun starts one rank per GPU on this host."""
    cmd = ["torchrun", "--nnodes", "1", "--nproc-per-node", str(n_ranks), "--master-addr", "127.0.0.1",
           "--master-port", str(master_port), script] + list(script_args) + ["--config-file", config_file]
    return "#!/bin/bash\n\n" + " ".join(shlex.quote(c) for c in cmd) + "\nwait\n"


def prepare(out_dir, n_gpus=None, script="main.py", script_args=(), **config_kw):
    """prepare.py:44-48 for a GPU node: dpwa.yaml with one node per GPU and an executable
    run.sh.  Returns (config path, run.sh path)."""
    if n_gpus is None:
        import torch
        n_gpus = torch.cuda.device_count()        # counts devices without initialising them
    if n_gpus < 1:
        raise ValueError("no GPUs to place nodes on")
    os.makedirs(out_dir, exist_ok=True)
    names = ["w%d" % g for g in range(n_gpus)]      # prepare.py:20 names nodes w<core>
    cfg = write_config(os.path.join(out_dir, "dpwa.yaml"), names, gpus=list(range(n_gpus)), **config_kw)
    run = os.path.join(out_dir, "run.sh")
    with open(run, "w") as f:
        f.write(run_script_text(n_gpus, script, script_args, "./dpwa.yaml"))
    os.chmod(run, os.stat(run).st_mode | stat.S_IEXEC)
    return cfg, run


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m dpwa_amd.launch")
    sub = ap.add_subparsers(dest="cmd", required=True)

    def config_opts(p):
        p.add_argument("--fetch-probability", type=float, default=1.0)
        p.add_argument("--timeout-ms", type=int, default=2500)
        p.add_argument("--interpolation", default="constant")
        p.add_argument("--divergence-threshold", type=float, default=0.0)
        p.add_argument("--constant-value", type=float, default=0.5)
        p.add_argument("--seed", type=int, default=None)

    mk = sub.add_parser("make-config", help="write a node list (one node per GPU rank)")
    mk.add_argument("--nodes", type=int, required=True)
    mk.add_argument("--out", required=True)
    mk.add_argument("--prefix", default="w")
    mk.add_argument("--gpus", type=int, default=None, help="add gpu: keys, nodes dealt round-robin over this many")
    config_opts(mk)
    pr = sub.add_parser("prepare", help="dpwa.yaml + run.sh for this host's GPUs (prepare.py for MI355X)")
    pr.add_argument("--gpus", type=int, default=None, help="default: every visible GPU")
    pr.add_argument("--out-dir", default=".")
    pr.add_argument("--script", default="main.py")
    config_opts(pr)
    argv = list(sys.argv[1:] if argv is None else argv)
    script_args = []
    if "--" in argv:
        i = argv.index("--")
        argv, script_args = argv[:i], argv[i + 1:]
    args = ap.parse_args(argv)
    fp = int(args.fetch_probability) if args.fetch_probability == 1 else args.fetch_probability
    kw = dict(fetch_probability=fp, timeout_ms=args.timeout_ms, interpolation=args.interpolation,
              divergence_threshold=args.divergence_threshold, constant_value=args.constant_value, seed=args.seed)
    if args.cmd == "make-config":
        names = ["%s%d" % (args.prefix, i + 1) for i in range(args.nodes)]
        gpus = None if args.gpus is None else [i % args.gpus for i in range(args.nodes)]
        write_config(args.out, names, gpus=gpus, **kw)
        print(args.out)
    else:
        cfg, run = prepare(args.out_dir, args.gpus, args.script, script_args, **kw)
        print(cfg)
        print(run)
    return 0


if __name__ == "__main__":
    sys.exit(main())
