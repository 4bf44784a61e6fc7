#!/bin/bash
# Round 4, final tree: clean one-GPU rehearsals of the driver's N>1 line over gloo (self-launched):
# N=2 and N=8 (the -m gpu suite ran in tools/gpu_final_r03.sh r04final), then the N=1 line.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r04m.sh <tag>
set -o pipefail
TAG=${1:-r04m}
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in ${NS:-2 8}; do
  t0=$(date +%s)
  timeout -k 10 600 python -u bench.py --gpus $N --dist-backend gloo --dist-sweep-max-numel 100000000 --steps 20 \
      --warmup 5 --no-cpu-baseline > gpurun_out/rh_${TAG}_n$N.json 2> gpurun_out/rh_${TAG}_n$N.err
  rc=$?
  echo "n$N rc=$rc $(( $(date +%s) - t0 ))s, stdout lines: $(wc -l < gpurun_out/rh_${TAG}_n$N.json)"
  [ $rc = 0 ] || { tail -20 gpurun_out/rh_${TAG}_n$N.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/rh_${TAG}_n$N.json'))
print(d.get('value'), d.get('pull_choice'), all(v for k,v in d['parity'].items() if k!='workload'), d.get('warmup_rounds'))
print(json.dumps(d.get('xgmi'))); print(json.dumps(d.get('reference_loop'))); print(json.dumps(d.get('overlap',{}).get('publish')), d.get('secondary_publish',{}).get('value'))
" || exit 1
done
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_n1.json 2> gpurun_out/bench_${TAG}_n1.err || { tail -20 gpurun_out/bench_${TAG}_n1.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_${TAG}_n1.json'));r=d['roofline']
print('n1', d['value'], r['achieved'], r['frac'], r['bytes_per_launch'], json.dumps(r['hbm']), r['avg_launch_us'], r['in_loop']['avg_launch_us'], list(d)[-1])" || exit 1
