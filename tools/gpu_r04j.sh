#!/bin/bash
# Round 4: does the N=1 pair loop need a longer warmup (clocks)?  bench at the driver's flags with
# --warmup-s 0.25 / 1 / 3, interleaved, twice.
set -o pipefail
TAG=${1:-r04j}
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
  for W in 3 0.25 1; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --warmup-s $W --no-cpu-baseline --no-sweep --compute-us 0 \
        --no-secondary > gpurun_out/warm_${TAG}_${W}_$pass.json 2> gpurun_out/warm_${TAG}_${W}_$pass.err || { tail gpurun_out/warm_${TAG}_${W}_$pass.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/warm_${TAG}_${W}_$pass.json'));r=d['roofline']
print('warmup_s $W pass $pass value',d['value'],'ms',d['ms_per_step'],'extra',d['warmup_rounds']['time_based_extra'],'cold',r['avg_launch_us'],'inloop',r['in_loop']['avg_launch_us'])"
  done
done
