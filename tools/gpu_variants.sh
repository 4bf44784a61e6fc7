#!/bin/bash
# Several run-time variants of the default bench line, interleaved over passes.
# Usage: gpurun -- bash tools/gpu_variants.sh <tag> <passes> "<ENV1>" "<ENV2>" ... [-- bench args]
set -o pipefail
TAG=$1; PASSES=$2; shift 2
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 $PASSES); do
  k=0
  for envs in "${VARS[@]}"; do
    k=$((k+1))
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ${VAR_SWEEP:---no-sweep} --compute-us 0 "$@" \
        > gpurun_out/var_${TAG}_v${k}_$i.json 2> gpurun_out/var_${TAG}_v${k}_$i.err || { echo "bench v$k/$i failed"; tail gpurun_out/var_${TAG}_v${k}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/var_${TAG}_v${k}_$i.json'));r=d['roofline'];print('pass $i', '$envs', 'value',d['value'],'ms',d['ms_per_step'],'inloop_us',r['in_loop']['avg_launch_us'],'cold_us',r['avg_launch_us'],'frac',r['frac'],'sizes',[(x['numel'],x['publish'],x['learners_per_launch'],x['frac']) for x in r.get('size_sweep',[])],'rounds',[x['value'] for x in d.get('round_sweep',[])])"
  done
done
