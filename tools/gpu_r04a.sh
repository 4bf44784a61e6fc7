#!/bin/bash
# Round 4: the changed suites, then one bench line (no CPU baseline).
# Usage: gpurun -- bash tools/gpu_r04a.sh <tag>
set -o pipefail
TAG=${1:-r04a}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_resident.py tests/test_gpu_timeout.py tests/test_gpu_gossip.py \
    > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -40; tail -3 gpurun_out/pytest_$TAG.log
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value',d['value'],'frac',d['roofline']['frac'])
print(json.dumps(d.get('reference_loop')))
print(json.dumps(d.get('overlap')))
print(list(d.keys())[-3:])
"
