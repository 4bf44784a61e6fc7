#!/usr/bin/env python3
"""Per-launch HBM traffic of the averaging kernel from rocprofv3 PMC passes.

Run (on the GPU box), one counter group per pass as MI355X_MICROARCH.md prescribes:
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py ...
then:
  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --out profiles/traffic_r01.json

FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts exactly half of the bytes
of a wide (16 B/lane) coalesced streaming read (TCC_EA0_RDREQ x 64 B for 128-B requests), so
it is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores (MI355X_MICROARCH.md §HBM).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def load(dirname, counter, kernel_substr):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no *counter_collection.csv under %s" % dirname)
    per_dispatch = {}
    names = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                if kernel_substr not in name:
                    continue
                d = (fn, row.get("Dispatch_Id"))
                per_dispatch[d] = per_dispatch.get(d, 0.0) + float(row["Counter_Value"])
                names[d] = name
    return per_dispatch, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--kernel", default="k_lerp<dpwa::OpsF32, 2, false,")
    ap.add_argument("--numel", type=int, default=11_173_962)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--publish", choices=["full", "write-through", "resident", "resident-pair"], default="full",
                    help="write-through: the kernel also writes the next snapshot (4*N*s algorithmic bytes); "
                         "resident-pair: two resident learners averaging with each other (4*N*s for both)")
    ap.add_argument("--learners", type=int, default=1, help="averages per dispatch (k_lerp_batch)")
    ap.add_argument("--basis", choices=["cold", "in-loop"], default="cold",
                    help="what the profiled command ran: tools/cold_sweep.py (cold) or bench.py's loop")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    fetch, names = load(args.fetch_dir, "FETCH_SIZE", args.kernel)
    write, _ = load(args.write_dir, "WRITE_SIZE", args.kernel)
    if not fetch or not write:
        raise SystemExit("no dispatches of %r found" % args.kernel)
    f_kib = statistics.median(fetch.values())
    w_kib = statistics.median(write.values())
    read_bytes = 2 * f_kib * 1024      # gfx950 FETCH_SIZE = 1/2 of 16-B/lane streaming reads
    write_bytes = w_kib * 1024
    esize = 4 if args.dtype == "f32" else 2
    algo = (4 * args.numel * esize if args.publish == "resident-pair" else
            args.learners * (4 if args.publish == "write-through" else 3) * args.numel * esize)
    out = {
        "kernel": sorted(set(names.values()))[0],
        "numel": args.numel,
        "dtype": args.dtype,
        "gpus": args.gpus,
        "publish": args.publish,
        "learners_per_launch": args.learners,
        "basis": args.basis,
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib,
        "hbm_read_bytes_per_launch": round(read_bytes),
        "hbm_write_bytes_per_launch": round(write_bytes),
        "hbm_bytes_per_launch": round(read_bytes + write_bytes),
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": round((read_bytes + write_bytes) / algo, 4),
        "correction": "FETCH_SIZE x 2 (gfx950, 16 B/lane loads); WRITE_SIZE exact",
    }
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
