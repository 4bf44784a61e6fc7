#!/bin/bash
# A/B of DPWA_LERP_POLICY=16 (only the write-through snapshot stored nt) against the product
# policy on the default bench loop, interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V="--no-cpu-baseline --no-sweep --compute-us 0 --steps 400 --warmup 40"
for i in 1 2 3; do
  for p in 0 16; do
    DPWA_LERP_POLICY=$p timeout -k 10 120 python bench.py $V > gpurun_out/pol_${p}_$i.json 2> gpurun_out/pol_${p}_$i.err || { echo "bench policy=$p failed"; tail gpurun_out/pol_${p}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/pol_${p}_$i.json')); r=d['roofline']; print('policy=$p run $i', d['value'], d['ms_per_step'], r['in_loop']['avg_launch_us'], r['avg_launch_us'], d['parity'].get('local'))"
  done
done
