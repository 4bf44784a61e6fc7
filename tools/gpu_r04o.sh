#!/bin/bash
# Round 4: the driver's N=1 bench command twice on one box (run-to-run spread of the final line).
set -o pipefail
TAG=${1:-r04o}
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err \
    || { tail -20 gpurun_out/bench_${TAG}_$i.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench_${TAG}_$i.json'));r=d['roofline']
print('run $i', d['value'], d['ms_per_step'], r['frac'], r['hbm']['frac'], r['avg_launch_us'], r['in_loop']['avg_launch_us'], [x['value'] for x in d['round_sweep']], d['reference_loop']['value'])" || exit 1
done
