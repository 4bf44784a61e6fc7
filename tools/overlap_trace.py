#!/usr/bin/env python3
"""f1 evidence: the gossip pull runs on the learner's side stream while the training step
runs on the compute stream (reference loop examples/pytorch-cifar/main.py:
122-158).

Default: two learners in one process on the box's one GPU, each training the CIFAR ResNet-18
of examples/resnet18_gossip.py on synthetic batches through DpwaPyTorchAdapter, in a
LocalGroup(prefetch=True, zero_copy=False): once both have published the round, each pull
(the copy kernel `k_pull` of the peer's snapshot into staging) starts on the learner's side
stream, then the forward/backward/SGD steps are enqueued on the compute stream and
update_wait averages.  This is the schedule of learners on different GPUs of one process
(peer-to-peer pulls over xGMI) and of one rank per GPU (`--procs 2`: the production
free-running group by default -- no barrier, the pull starts at update_send on the side
stream; `--gossip lockstep` uses DistGroup, whose gloo barrier on one GPU synchronises the
host every round, so there the pull finishes before the host has enqueued the step).  Run it under

  rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/overlap -o ov -- python3 tools/overlap_trace.py

and then `python3 tools/overlap_trace.py --analyze gpurun_out/overlap` reports, per process,
how much of each pull's execution overlapped that same process's training kernels.
"""
import argparse
import csv
import glob
import json
import os
import socket
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, world, port, cfg, steps, batch, out_dir, gossip="async", sync_loss=True):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import time

    import torch
    import torch.distributed as dist
    import torch.nn.functional as F
    from resnet18_gossip import resnet18

    from dpwa_amd import DpwaPyTorchAdapter
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(rank)
    net = resnet18().to(dev)
    adapter = DpwaPyTorchAdapter(net, "w%d" % rank, cfg, seed=100 + rank, group=gossip, pull="kernel:256")
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    x = torch.randn(batch, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (batch,), device=dev)

    host = {"send": 0.0, "wait": 0.0, "n": 0, "sends": [], "waits": []}

    def step(gossip, loss):
        if gossip:
            t = time.perf_counter()
            adapter.update_send(loss)
            host["send"] += time.perf_counter() - t
            host["sends"].append(time.perf_counter() - t)
        opt.zero_grad(set_to_none=True)
        out = F.cross_entropy(net(x), y)
        out.backward()
        opt.step()
        # main.py:142 reads the loss on the host every step (a sync), and passes a float
        loss = float(out) if sync_loss else out.detach()
        if gossip:
            t = time.perf_counter()
            adapter.update_wait(loss)
            host["wait"] += time.perf_counter() - t
            host["waits"].append(time.perf_counter() - t)
            host["n"] += 1
        return loss

    loss = 2.3 if sync_loss else torch.tensor(2.3, device=dev)
    times = {}
    sequence = []
    for gossip in (False, True) * 3:      # interleaved: the first phase runs at a higher clock
        for _ in range(5):
            loss = step(gossip, loss)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = step(gossip, loss)
        torch.cuda.synchronize()
        times[gossip] = time.perf_counter() - t0
        sequence.append(("gossip" if gossip else "plain", round(1e3 * times[gossip] / steps, 3)))
        dist.barrier()
    with open(os.path.join(out_dir, "overlap_rank%d.json" % rank), "w") as f:
        json.dump({"rank": rank, "pid": os.getpid(), "steps": steps, "batch": batch,
                   "ms_per_step_plain": 1e3 * times[False] / steps, "ms_per_step_gossip": 1e3 * times[True] / steps,
                   "final_clock": adapter.connection.clock, "sequence_ms_per_step": sequence,
                   "host_ms_in_update_send": 1e3 * host["send"] / max(1, host["n"]),
                   "host_ms_in_update_wait": 1e3 * host["wait"] / max(1, host["n"]),
                   "host_ms_update_send_median_max": [round(1e3 * sorted(host["sends"])[len(host["sends"]) // 2], 3),
                                                      round(1e3 * max(host["sends"]), 3)] if host["sends"] else None},
                  f)
    adapter.connection.close()
    dist.barrier()
    dist.destroy_process_group()


def run_local(args):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import time

    import torch
    import torch.nn.functional as F
    from resnet18_gossip import resnet18

    from dpwa_amd import DpwaPyTorchAdapter
    from dpwa_amd.group import LocalGroup
    from dpwa_amd.launch import write_config
    tmp = tempfile.mkdtemp(prefix="dpwa_overlap_")
    cfg = write_config(os.path.join(tmp, "dpwa.yaml"), ["w0", "w1"], interpolation="constant")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    nets = [resnet18().to(dev) for _ in range(2)]
    group = LocalGroup(prefetch=True, zero_copy=False)
    adapters = [DpwaPyTorchAdapter(n, "w%d" % i, cfg, seed=100 + i, group=group, pull="kernel:256")
                for i, n in enumerate(nets)]
    opts = [torch.optim.SGD(n.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4) for n in nets]
    x = torch.randn(args.batch, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (args.batch,), device=dev)
    losses = [torch.tensor(2.3, device=dev) for _ in nets]

    def step(gossip):
        if gossip:
            for a, l in zip(adapters, losses):
                a.update_send(l)
        for i, (n, o) in enumerate(zip(nets, opts)):
            o.zero_grad(set_to_none=True)
            out = F.cross_entropy(n(x), y)
            out.backward()
            o.step()
            losses[i] = out.detach()
        if gossip:
            for a, l in zip(adapters, losses):
                a.update_wait(l)

    times = {}
    for gossip in (False, True):
        for _ in range(5):
            step(gossip)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(gossip)
        torch.cuda.synchronize()
        times[gossip] = time.perf_counter() - t0
    print(json.dumps({"learners": 2, "process": os.getpid(), "steps": args.steps, "batch": args.batch,
                      "ms_per_step_plain": 1e3 * times[False] / args.steps,
                      "ms_per_step_gossip": 1e3 * times[True] / args.steps,
                      "gossip_overhead_pct": 100.0 * (times[True] / times[False] - 1.0),
                      "final_clock": adapters[0].connection.clock}))
    for a in adapters:
        a.connection.close()


def run(args):
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    from dpwa_amd.launch import write_config
    tmp = tempfile.mkdtemp(prefix="dpwa_overlap_")
    cfg = write_config(os.path.join(tmp, "dpwa.yaml"), ["w0", "w1"], interpolation="constant",
                       fetch_probability=args.fetch_probability)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.makedirs(args.out, exist_ok=True)
    mp.spawn(worker, args=(2, port, cfg, args.steps, args.batch, args.out, args.gossip, not args.no_sync),
             nprocs=2, join=True)
    res = [json.load(open(os.path.join(args.out, "overlap_rank%d.json" % r))) for r in range(2)]
    print(json.dumps(res))


def analyze(trace_dir):
    """Per process: the share of k_pull's execution time during which a kernel of the same
    process's training step (anything other than dpwa's own and the pull) was running."""
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((fn, r))
    by_proc = {}
    for fn, r in rows:
        key = (fn, r.get("Agent_Id"))
        by_proc.setdefault(fn, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                                           r.get("Stream_Id", ""), r.get("Queue_Id", "")))
        del key
    out = []
    for fn, ks in by_proc.items():
        pulls = [k for k in ks if "k_pull" in k[2]]
        train = [k for k in ks if "dpwa::" not in k[2] and "spin_kernel" not in k[2]]
        if not pulls:
            continue
        covered = total = 0
        overlapped_pulls = 0
        for s0, e0, _, _, _ in pulls:
            segs = sorted((max(s0, s), min(e0, e)) for s, e, _, _, _ in train if s < e0 and e > s0)
            cov, cur = 0, s0
            for a, b in segs:
                a = max(a, cur)
                if b > a:
                    cov += b - a
                    cur = b
            covered += cov
            total += e0 - s0
            overlapped_pulls += cov > 0
        out.append({"trace": os.path.relpath(fn, trace_dir), "pulls": len(pulls), "pulls_overlapping_training": overlapped_pulls,
                    "pull_time_overlapped_frac": round(covered / max(1, total), 4),
                    "avg_pull_us": round(total / len(pulls) / 1e3, 2), "training_kernels": len(train)})
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "overlap_runs"))
    ap.add_argument("--procs", type=int, default=1, choices=[1, 2],
                    help="1: two learners in this process (prefetching LocalGroup); 2: one rank each")
    ap.add_argument("--fetch-probability", type=float, default=1.0, help="--procs 2: the config's fetch_probability")
    ap.add_argument("--no-sync", action="store_true",
                    help="--procs 2: keep the loss on the device (the reference loop reads it every step)")
    ap.add_argument("--gossip", default="async", choices=["async", "lockstep"],
                    help="--procs 2: free-running rounds (the default group, no per-round barrier) or lock-step")
    ap.add_argument("--analyze", default=None, help="rocprofv3 output directory to analyse instead of running")
    args = ap.parse_args()
    if args.analyze:
        analyze(args.analyze)
    elif args.procs == 1:
        run_local(args)
    else:
        run(args)


if __name__ == "__main__":
    main()
