#!/bin/bash
# Round 4: the time-based warmup A/B at the driver's flags, then the evidence script.
set -o pipefail
TAG=${1:-r04h}
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
  for W in 0.25 0; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --warmup-s $W --no-cpu-baseline --no-sweep --compute-us 0 \
        > gpurun_out/warm_${TAG}_${W}_$pass.json 2> gpurun_out/warm_${TAG}_${W}_$pass.err || { tail gpurun_out/warm_${TAG}_${W}_$pass.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/warm_${TAG}_${W}_$pass.json'));r=d['roofline']
print('warmup_s $W pass $pass value',d['value'],'ms',d['ms_per_step'],'extra',d['warmup_rounds']['time_based_extra'],'cold',r['avg_launch_us'],'inloop',r['in_loop']['avg_launch_us'])"
  done
done
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 5 --warmup-s 0 --no-cpu-baseline --no-sweep --compute-us 0 \
    > gpurun_out/warm_${TAG}_long.json 2> gpurun_out/warm_${TAG}_long.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/warm_${TAG}_long.json'));print('2000 steps, no time warmup: value',d['value'],'ms',d['ms_per_step'])"
bash tools/gpu_evidence_r04.sh $TAG
