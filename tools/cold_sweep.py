#!/usr/bin/env python3
"""The averaging kernel alone, cold (bench.cold_kernel), for profiling: every launch of the
product kernel over rotating buffers, nothing else on the GPU, so a rocprofv3 kernel trace or
PMC pass of this command sees only cold launches of that kernel.

  python tools/cold_sweep.py                                  # configs[1]: 11.17M fp32, both publish forms
  python tools/cold_sweep.py --sizes 11173962:f32 --publish write-through
  python tools/cold_sweep.py --publish write-through --learners 2     # the batched dispatch of N=1
  python tools/cold_sweep.py --publish resident --learners 2          # ... of resident learners
  rocprofv3 --kernel-trace --stats -d gpurun_out/cold -o c -- python3 tools/cold_sweep.py --all
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="%d:f32" % bench.RESNET18_NUMEL,
                    help="comma-separated numel:dtype list (dtype f32 or bf16)")
    ap.add_argument("--all", action="store_true", help="every north_star size (bench.SWEEP)")
    ap.add_argument("--publish", choices=["full", "write-through", "resident", "resident-pair", "both", "all"],
                    default="both", help="resident-pair (with --learners 2): the N=1 loop's mutual pair, 4*N*s")
    ap.add_argument("--launches", type=int, default=64)
    ap.add_argument("--learners", type=int, default=1,
                    help="averages per dispatch: 1 = dpwa_average (k_lerp), > 1 = dpwa_average_many (k_lerp_batch, "
                         "the N=1 loop's kernel)")
    args = ap.parse_args()
    sizes = [(n, d) for n, d in bench.SWEEP] if args.all else \
        [(int(x.split(":")[0]), x.split(":")[1]) for x in args.sizes.split(",")]
    forms = {"full": ["full"], "write-through": ["write-through"], "resident": ["resident"],
             "resident-pair": ["resident-pair"],
             "both": ["full", "write-through"], "all": ["full", "write-through", "resident"]}[args.publish]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for numel, dt in sizes:
        dtype = torch.float32 if dt == "f32" else torch.bfloat16
        esize = 4 if dt == "f32" else 2
        for form in forms:
            wt = form == "write-through"
            pair = form == "resident-pair"
            c = bench.cold_kernel(numel, dtype, dev, wt, args.launches, learners=args.learners,
                                  resident=form.startswith("resident"), pair=pair)
            nbytes = 4 * numel * esize if pair else args.learners * (4 if wt else 3) * numel * esize
            gbs = nbytes / (c["avg_launch_us"] * 1e-6) / 1e9
            print(json.dumps(dict(numel=numel, dtype=dt, publish=form,
                                  bytes_per_launch=nbytes, achieved=round(gbs, 1),
                                  frac=round(gbs / bench.HBM_PEAK_GBS, 4),
                                  **{k: (round(v, 2) if isinstance(v, float) else v) for k, v in c.items()})),
                  flush=True)


if __name__ == "__main__":
    main()
