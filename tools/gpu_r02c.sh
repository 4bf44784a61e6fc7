#!/bin/bash
# Store-policy A/B of the averaging kernel inside the bench loop and cold (DPWA_LERP_POLICY),
# then the cold sweep under rocprofv3 (kernel trace + stats).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --no-sweep --compute-us 0 --no-parity --steps 300 --warmup 30"
for i in 1 2; do
  for pol in ${POLICIES:-0 4 5}; do
    DPWA_LERP_POLICY=$pol timeout -k 10 180 python3 $B > gpurun_out/pol${pol}_$i.json 2> gpurun_out/pol${pol}_$i.err \
      || { echo "bench policy $pol failed"; tail -20 gpurun_out/pol${pol}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/pol${pol}_$i.json'));r=d['roofline'];s=d['secondary_publish'];print('pol $pol', d['value'], d['ms_per_step'], 'cold', r['avg_launch_us'], r['frac'], 'loop', r['in_loop']['avg_launch_us'], 'full', s['value'], s['avg_launch_us'])"
  done
done
[ -n "$NO_COLD_PROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cold_prof -o cold -- \
    python3 tools/cold_sweep.py --all > gpurun_out/cold_sweep.jsonl 2> gpurun_out/cold_sweep.err \
    || { echo "cold sweep failed"; tail -20 gpurun_out/cold_sweep.err; exit 1; }
cat gpurun_out/cold_sweep.jsonl
