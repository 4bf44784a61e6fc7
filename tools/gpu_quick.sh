#!/bin/bash
# Quick GPU pass: host cost per round, then the bench line at the driver's flags (CPU baseline
# optional: QUICK_CPU=1 keeps it).  Usage: gpurun -- bash tools/gpu_quick.sh <tag> [bench args]
set -o pipefail
TAG=${1:-quick}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/host_overhead.py > gpurun_out/host_$TAG.json 2> gpurun_out/host_$TAG.err \
    || { echo "host overhead failed"; tail gpurun_out/host_$TAG.err; exit 1; }
cat gpurun_out/host_$TAG.json
CPUF="--no-cpu-baseline"; [ "${QUICK_CPU:-0}" = 1 ] && CPUF=""
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 $CPUF "$@" > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err \
      || { echo "bench failed"; tail gpurun_out/bench_${TAG}_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$i.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'frac',r['frac'],'inloop_us',r['in_loop']['avg_launch_us'],'sweep11',d.get('round_sweep',[{}])[0].get('value'))"
done
