#!/bin/bash
# A/B of a run-time knob on the default bench line, interleaved ABAB...: each pass runs
# bench.py at the driver's flags (no CPU baseline) once with ENV_A and once with ENV_B.
# Usage: gpurun -- bash tools/gpu_ab.sh <tag> "<ENV_A>" "<ENV_B>" [pairs] [bench args...]
set -o pipefail
TAG=$1; A=$2; B=$3; PAIRS=${4:-3}; shift 4
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 $PAIRS); do
  for side in A B; do
    envs=$A; [ $side = B ] && envs=$B
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" \
        > gpurun_out/ab_${TAG}_${side}$i.json 2> gpurun_out/ab_${TAG}_${side}$i.err || { echo "bench $side$i failed"; tail gpurun_out/ab_${TAG}_${side}$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_${side}$i.json'));r=d['roofline'];print('$side$i', '$envs', 'value',d['value'],'ms',d['ms_per_step'],'inloop_us',r['in_loop']['avg_launch_us'],'cold_us',r['avg_launch_us'],'sweep',[x['value'] for x in d.get('round_sweep',[])])"
  done
done
