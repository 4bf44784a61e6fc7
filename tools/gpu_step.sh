#!/bin/bash
# One GPU pass of this round: a pytest selection, then a bench line with the driver's flags.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_step.sh <tag> "<pytest selection>" ["<bench args>"]
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-step}
SEL=${2:-tests}
BARGS=${3:---steps 20 --warmup 5}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$SEL" != "none" ]; then
  timeout -k 10 800 python -u -m pytest $SEL -m gpu -v -x --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu_$TAG.log | tail -5
  tail -3 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 1; fi
fi
if [ "$BARGS" != "none" ]; then
  timeout -k 10 900 python -u bench.py $BARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?
  tail -5 gpurun_out/bench_$TAG.err
  if [ $rc -ne 0 ]; then echo "bench rc=$rc"; exit 1; fi
  python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'frac',r['frac'],'us',r['avg_launch_us'],'inloop',r['in_loop']['frac'],r['in_loop']['avg_launch_us'])"
fi
