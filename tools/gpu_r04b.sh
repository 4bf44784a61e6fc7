#!/bin/bash
# Round 4: the whole -m gpu suite, then clean one-GPU rehearsals of the driver's N>1 line over gloo
# (self-launched, secondary publish form and overlap on): N=2 and N=8.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r04b.sh <tag>
set -o pipefail
TAG=${1:-r04b}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -20; tail -3 gpurun_out/pytest_$TAG.log
[ $rc = 0 ] || exit $rc
for N in 2 8; do
  t0=$(date +%s)
  timeout -k 10 600 python -u bench.py --gpus $N --dist-backend gloo --dist-sweep-max-numel 100000000 --steps 20 \
      --warmup 5 --no-cpu-baseline > gpurun_out/rh_${TAG}_n$N.json 2> gpurun_out/rh_${TAG}_n$N.err
  echo "n$N rc=$? $(( $(date +%s) - t0 ))s, stdout lines: $(wc -l < gpurun_out/rh_${TAG}_n$N.json)"
  python3 -c "
import json;d=json.load(open('gpurun_out/rh_${TAG}_n$N.json'))
print(d.get('value'), d.get('pull_choice'), all(v for k,v in d['parity'].items() if k!='workload'))
print(json.dumps(d.get('xgmi'))); print(json.dumps(d.get('reference_loop'))); print(json.dumps(d.get('overlap',{}).get('publish')), d.get('secondary_publish',{}).get('value'))
" || exit 1
done
timeout -k 10 180 tools/stream_tune 11173962 12 > gpurun_out/stream_tune_${TAG}_11m.log 2>&1 || exit 1
grep -E "oop|dual|copy" gpurun_out/stream_tune_${TAG}_11m.log
