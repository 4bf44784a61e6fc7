#!/bin/bash
# Round 4: k_lerp_duo (two equal-size in-place averages in one workgroup per span: the N=1 reference
# loop's write-through pair): the batch / gossip / pair suites, then the bench with it on and off
# (DPWA_DUO=0: the batched kernel), interleaved; reference_loop is the write-through figure.
set -o pipefail
TAG=${1:-r04t}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py \
    tests/test_gpu_pairs.py tests/test_gpu_gossip.py > gpurun_out/pytest_$TAG.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for pass in 1 2; do
  for f in 1 0; do
    DPWA_DUO=$f timeout -k 10 600 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep \
        > gpurun_out/bench_${TAG}_d${f}_$pass.json 2> gpurun_out/bench_${TAG}_d${f}_$pass.err \
        || { tail -20 gpurun_out/bench_${TAG}_d${f}_$pass.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/bench_${TAG}_d${f}_$pass.json'));r=d['reference_loop'];s=d.get('secondary_publish',{})
print('duo=$f pass $pass', 'ref', r['value'], r['ms_per_step'], json.dumps(r['kernel_cold']), 'sec', s.get('value'), 'main', d['value'])" || exit 1
  done
done
