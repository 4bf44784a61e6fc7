#!/bin/bash
# Round 4: the fused mutual-pair kernel (k_lerp_pair): parity suites, then the bench with it on and
# off (DPWA_PAIR_FUSED=0: the XCD-grouped batch), interleaved.
set -o pipefail
TAG=${1:-r04q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pairs.py \
    tests/test_gpu_batch.py tests/test_gpu_resident.py "tests/test_gpu_configs.py::test_full_size_configs_resident" \
    > gpurun_out/pytest_$TAG.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for pass in 1 2; do
  for f in 1 0; do
    DPWA_PAIR_FUSED=$f timeout -k 10 600 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline \
        > gpurun_out/bench_${TAG}_f${f}_$pass.json 2> gpurun_out/bench_${TAG}_f${f}_$pass.err \
        || { tail -20 gpurun_out/bench_${TAG}_f${f}_$pass.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/bench_${TAG}_f${f}_$pass.json'));r=d['roofline']
print('fused=$f pass $pass', d['value'], d['ms_per_step'], 'cold', r['avg_launch_us'], r['frac'], r['hbm']['frac'], 'inloop', r['in_loop']['avg_launch_us'], [x['value'] for x in d['round_sweep']], d['parity'])" || exit 1
  done
done
