#!/bin/bash
# Round 4: cache policies of k_lerp_pair (DPWA_LERP_POLICY), whole bench without sweeps, 200 steps,
# two interleaved passes.
set -o pipefail
TAG=${1:-r04u}
mkdir -p gpurun_out
for pass in 1 2; do
  for pol in 8 0 1 2 16 32; do
    DPWA_LERP_POLICY=$pol timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep \
        --no-secondary > gpurun_out/bench_${TAG}_p${pol}_$pass.json 2> gpurun_out/bench_${TAG}_p${pol}_$pass.err \
        || { tail -20 gpurun_out/bench_${TAG}_p${pol}_$pass.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/bench_${TAG}_p${pol}_$pass.json'));r=d['roofline']
print('policy $pol pass $pass', d['value'], 'cold', r['avg_launch_us'], r['hbm']['frac'], 'inloop', r['in_loop']['avg_launch_us'], d['parity'].get('local+res'))" || exit 1
  done
done
