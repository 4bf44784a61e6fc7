#!/usr/bin/env python3
"""Gossip training of a CIFAR-shaped ResNet-18 on synthetic data.

The caller of the hot path, as the reference's examples/pytorch-cifar/main.py:122-158 uses
it: ``update_send(loss)`` before the forward pass, ``update_wait(loss)`` after
``optimizer.step()``.  No dataset is downloaded: inputs are random 3x32x32 images with random
labels (torchvision/CIFAR are not available offline).

  python examples/resnet18_gossip.py --learners 2 --steps 50         # co-resident learners, 1 GPU
  torchrun --nproc-per-node 8 examples/resnet18_gossip.py --steps 50  # one learner per GPU

Prints one JSON line: training steps/s with and without gossip and the gossip overhead.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def conv_bn(cin, cout, stride):
    return nn.Sequential(nn.Conv2d(cin, cout, 3, stride, 1, bias=False), nn.BatchNorm2d(cout))


class Residual(nn.Module):
    """Two 3x3 conv-BN layers with an identity (or 1x1-projected) shortcut."""

    def __init__(self, cin, cout, stride):
        super().__init__()
        self.a = conv_bn(cin, cout, stride)
        self.b = conv_bn(cout, cout, 1)
        self.skip = (nn.Sequential() if stride == 1 and cin == cout else
                     nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout)))

    def forward(self, x):
        return F.relu(self.b(F.relu(self.a(x))) + self.skip(x))


def resnet18(num_classes=10):
    """CIFAR ResNet-18: 11,173,962 parameters (the reference's ResNet18(), models/resnet.py:102)."""
    widths, strides = (64, 128, 256, 512), (1, 2, 2, 2)
    layers = [conv_bn(3, 64, 1), nn.ReLU()]
    cin = 64
    for w, s in zip(widths, strides):
        layers += [Residual(cin, w, s), Residual(w, w, 1)]
        cin = w
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, num_classes)]
    return nn.Sequential(*layers)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--learners", type=int, default=2, help="co-resident learners (single process)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=8)      # prepare.py:31
    ap.add_argument("--lr", type=float, default=0.01)         # prepare.py:31
    ap.add_argument("--interpolation", default="constant")
    ap.add_argument("--gossip", default="async", choices=["lockstep", "async"],
                    help="under torchrun: lock-step rounds (DistGroup) or free-running ones (gossip board)")
    ap.add_argument("--pull", default=None,
                    help="under torchrun: copy | kernel[:blocks] | relay[:blocks] | relay-avg[:blocks] "
                         "(the relays need --gossip lockstep)")
    ap.add_argument("--no-batch-wait", dest="batch_wait", action="store_false",
                    help="co-resident learners: one update_wait per adapter instead of update_wait_many")
    ap.add_argument("--resident", action="store_true",
                    help="resident parameters (the adapter's resident=True): the loop runs update_send, "
                         "update_wait, then the training step -- nothing may write the parameters between "
                         "update_send and update_wait in this form -- instead of the reference's update_send, "
                         "step, update_wait")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    from dpwa_amd import DpwaPyTorchAdapter
    from dpwa_amd.launch import write_config

    n_nodes = world if world > 1 else args.learners
    names = ["w%d" % (i + 1) for i in range(n_nodes)]
    cfg = os.path.join(tempfile.mkdtemp(), "dpwa.yaml")
    write_config(cfg, names, interpolation=args.interpolation, divergence_threshold=0.5)
    mine = [rank] if world > 1 else list(range(n_nodes))
    torch.manual_seed(0)
    nets = [resnet18().to(dev) for _ in mine]
    assert sum(p.numel() for p in nets[0].parameters()) == 11_173_962
    opts = [torch.optim.SGD(n.parameters(), lr=args.lr, momentum=0.9, weight_decay=5e-4) for n in nets]
    x = torch.randn(args.batch_size, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (args.batch_size,), device=dev)

    def train_step(i):
        opts[i].zero_grad(set_to_none=True)
        loss = F.cross_entropy(nets[i](x), y)
        loss.backward()
        opts[i].step()
        return loss.detach()

    def run(steps, gossip, adapters=None):
        losses = [torch.tensor(2.3, device=dev) for _ in mine]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            if gossip:
                for i, a in enumerate(adapters):
                    a.update_send(losses[i])       # a device tensor: no host sync
            if not args.resident:                  # the reference's order (README.md:18-29)
                for i in range(len(mine)):
                    losses[i] = train_step(i)
            if gossip:
                if len(adapters) > 1 and args.batch_wait:    # co-resident: one averaging dispatch
                    DpwaPyTorchAdapter.update_wait_many(adapters, losses)
                else:
                    for i, a in enumerate(adapters):
                        a.update_wait(losses[i])
            if args.resident:                      # resident parameters: the step after update_wait
                for i in range(len(mine)):
                    losses[i] = train_step(i)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    group = {"group": args.gossip} if world > 1 else {}
    if world > 1 and args.pull:
        group["pull"] = args.pull
    adapters = [DpwaPyTorchAdapter(nets[i], names[g], cfg, seed=100 + g, resident=args.resident, **group)
                for i, g in enumerate(mine)]
    run(args.warmup, False)
    run(args.warmup, True, adapters)
    # interleaved phases, the first pair discarded: a run's first phase executes at a higher
    # GPU clock than the later ones (profiles/r02_overlap_2proc.json)
    sequence = []
    for gossip in (False, True) * 3:
        sequence.append((gossip, run(args.steps, gossip, adapters)))
    t_plain = sum(t for g, t in sequence[2:] if not g) / 2
    t_gossip = sum(t for g, t in sequence[2:] if g) / 2
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([t_plain, t_gossip], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_plain, t_gossip = t.tolist()
    if rank == 0:
        print(json.dumps({
            "model": "ResNet-18 (CIFAR, 11,173,962 params), synthetic batch %d" % args.batch_size,
            "learners": n_nodes, "gpus": world,
            "train_steps_per_s_per_learner_plain": round(args.steps / t_plain, 1),
            "train_steps_per_s_per_learner_gossip": round(args.steps / t_gossip, 1),
            "gossip_overhead_pct": round(100 * (t_gossip - t_plain) / t_plain, 2),
            "batched_wait": bool(args.batch_wait and len(adapters) > 1),
            "resident": bool(args.resident),
            "final_clock": adapters[0].connection.clock,
        }))
    for a in adapters:
        a.connection.close()


if __name__ == "__main__":
    main()
