#!/bin/bash
# Resident parameters: their GPU tests (plus the batched-dispatch and gossip suites they build on),
# then the default bench line without the CPU baseline and sweeps.
# Usage: gpurun --timeout 900 -- bash tools/gpu_resident.sh <tag>
set -o pipefail
TAG=${1:-res}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_resident.py tests/test_gpu_batch.py > gpurun_out/pytest_$TAG.log 2>&1 \
    || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'frac',r['frac'],r['avg_launch_us'],'inloop',r['in_loop']['avg_launch_us'],r['in_loop']['frac'],'parity',d.get('parity'),'sec',d.get('secondary_publish',{}).get('value'))"
echo done
