#!/bin/bash
# Round 4: the XCD-paired mutual pairs -- parity (pairs, batch, resident suites), pair_tune, and a
# bench line with and without the pairing (DPWA_BATCH_SHARE=0).
set -o pipefail
TAG=${1:-r04g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_pairs.py tests/test_gpu_batch.py tests/test_gpu_resident.py > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_$TAG.log | head -20; tail -3 gpurun_out/pytest_$TAG.log
[ $rc = 0 ] || exit $rc
timeout -k 10 240 tools/pair_tune 11173962 12 > gpurun_out/pair_tune_${TAG}_11m.log 2>&1 || { cat gpurun_out/pair_tune_${TAG}_11m.log; exit 1; }
cat gpurun_out/pair_tune_${TAG}_11m.log
for P in 1 0 1 0; do
  DPWA_BATCH_SHARE=$P timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --compute-us 0 \
      > gpurun_out/bench_${TAG}_share$P.json 2> gpurun_out/bench_${TAG}_share$P.err || { tail gpurun_out/bench_${TAG}_share$P.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench_${TAG}_share$P.json'));r=d['roofline']
print('share=$P value',d['value'],'ms',d['ms_per_step'],'cold_us',r['avg_launch_us'],'inloop_us',r['in_loop']['avg_launch_us'],'rs',[x['value'] for x in d['round_sweep']])"
done
