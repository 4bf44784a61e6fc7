#!/bin/bash
# A/B of a sweep-direction knob (DPWA_LERP_ALTERNATE, since removed): consecutive
# averages of a learner sweeping in opposite directions.  Kept as the record of that experiment.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V="--no-cpu-baseline --no-sweep --no-cold --compute-us 0 --steps 400 --warmup 40"
for i in 1 2 3; do
  for a in 0 1; do
    DPWA_LERP_ALTERNATE=$a timeout -k 10 120 python bench.py $V > gpurun_out/alt_${a}_$i.json 2> gpurun_out/alt_${a}_$i.err || { echo "bench alt=$a failed"; tail gpurun_out/alt_${a}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/alt_${a}_$i.json')); print('alt=$a run $i', d['value'], d['ms_per_step'], d['roofline']['in_loop']['avg_launch_us'], d['secondary_publish']['value'], d['parity'].get('local'))"
  done
done
for n in 100000000; do
  for a in 0 1; do
    DPWA_LERP_ALTERNATE=$a timeout -k 10 200 python bench.py $V --numel $n --steps 60 --warmup 10 > gpurun_out/alt_${a}_100m.json 2>> gpurun_out/alt_100m.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/alt_${a}_100m.json')); print('100M alt=$a', d['value'], d['ms_per_step'], d['roofline']['in_loop']['avg_launch_us'])"
  done
done
DPWA_LERP_ALTERNATE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_seam.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/alt_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/alt_pytest.log; exit $rc
