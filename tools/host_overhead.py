#!/usr/bin/env python3
"""Host-side cost of one gossip round through the drop-in API (the part of a round a
host-bound training loop pays on the CPU): two learners in one process, a ResNet-18-shaped
parameter list (62 tensors) scaled down so the GPU work is negligible, timed per call with
time.perf_counter over many rounds.  Prints one JSON line (microseconds per call and learner;
connection_batched: both learners' update_wait in one update_wait_average_many call; the
_resident modes: resident learners -- the adapter re-points its 62 parameters every round, the
connection re-reads conn.parameters)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main(rounds=2000):
    from dpwa_amd import DpwaConnection, DpwaPyTorchAdapter
    from dpwa_amd.group import LocalGroup
    from dpwa_amd.launch import write_config
    from oracle.ref_round import resnet18_shapes
    dev = torch.device("cuda", 0)
    cfg = write_config(os.path.join(tempfile.mkdtemp(), "h.yaml"), ["a", "b"], interpolation="constant")

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            for i, s in enumerate(resnet18_shapes()):
                self.register_parameter("p%d" % i, torch.nn.Parameter(torch.zeros(min(64, int(torch.tensor(s).prod())))))

    out = {}
    for mode in ("adapter", "connection", "connection_batched", "adapter_resident", "adapter_resident_batched",
                 "connection_batched_resident"):
        group = LocalGroup()
        if mode.startswith("adapter"):
            nets = [Net().to(dev), Net().to(dev)]
            ads = [DpwaPyTorchAdapter(n, nm, cfg, seed=i, group=group, resident="resident" in mode)
                   for i, (n, nm) in enumerate(zip(nets, "ab"))]
            send = [a.update_send for a in ads]
            wait = [a.update_wait for a in ads]
            if mode.endswith("batched"):
                wait = [lambda l: DpwaPyTorchAdapter.update_wait_many(ads, [l, l])]
            conns = [a.connection for a in ads]
        elif mode == "connection_batched_resident":
            conns = [DpwaConnection(nm, cfg, seed=i, group=group) for i, nm in enumerate("ab")]
            for i, c in enumerate(conns):
                c.make_resident(torch.full((4096,), float(i), device=dev))
            cur = [c.parameters for c in conns]

            def _send(l, i):
                conns[i].update_send(cur[i], l)

            def _wait(l):
                DpwaConnection.update_wait_average_many(conns, cur, [l, l])
                cur[:] = [c.parameters for c in conns]
            send = [lambda l: _send(l, 0), lambda l: _send(l, 1)]
            wait = [_wait]
        else:
            flats = [torch.zeros(4096, device=dev), torch.ones(4096, device=dev)]
            conns = [DpwaConnection(nm, cfg, seed=i, group=group) for i, nm in enumerate("ab")]
            send = [lambda l, c=c, f=f: c.update_send(f, l, reuse_snapshot=True) for c, f in zip(conns, flats)]
            wait = [lambda l, c=c, f=f: c.update_wait_average(f, l, write_through=True) for c, f in zip(conns, flats)]
            if mode == "connection_batched":     # both averages in one call (and one dispatch)
                wait = [lambda l: DpwaConnection.update_wait_average_many(conns, flats, [l, l], write_through=True)]
        for loss_kind in ("float", "tensor"):
            loss = 1.0 if loss_kind == "float" else torch.tensor(1.0, device=dev)
            for _ in range(50):
                for s in send:
                    s(loss)
                for w in wait:
                    w(loss)
            torch.cuda.synchronize()
            ts = tw = 0.0
            for _ in range(rounds):
                t0 = time.perf_counter()
                for s in send:
                    s(loss)
                t1 = time.perf_counter()
                for w in wait:
                    w(loss)
                t2 = time.perf_counter()
                ts += t1 - t0
                tw += t2 - t1
                if _ % 64 == 0:
                    torch.cuda.synchronize()      # keep the GPU queue short
            torch.cuda.synchronize()
            out["%s/%s_loss" % (mode, loss_kind)] = {"update_send_us": round(1e6 * ts / (2 * rounds), 2),
                                                     "update_wait_us": round(1e6 * tw / (2 * rounds), 2),
                                                     "round_us_both_learners": round(1e6 * (ts + tw) / rounds, 2)}
        for c in conns:
            c.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
