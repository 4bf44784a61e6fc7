#!/bin/bash
# Round 4: store-scope A/B.  stream_tune twice at 11.17M and once at 100M, then bench.py with the
# product policy (8) and with sc0+sc1 stores (2), three interleaved pairs (no CPU baseline).
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r04c.sh <tag>
set -o pipefail
TAG=${1:-r04c}
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 180 tools/stream_tune 11173962 12 > gpurun_out/stream_tune_${TAG}_11m_$i.log 2>&1 || exit 1
done
timeout -k 10 300 tools/stream_tune 100000000 6 > gpurun_out/stream_tune_${TAG}_100m.log 2>&1 || exit 1
grep -E "oop|dual|avg  64x1" gpurun_out/stream_tune_${TAG}_11m_2.log
for pass in 1 2 3; do
  for P in 8 2 40 0; do
    DPWA_LERP_POLICY=$P timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --compute-us 0 \
        > gpurun_out/ab_${TAG}_p${P}_$pass.json 2> gpurun_out/ab_${TAG}_p${P}_$pass.err || { tail gpurun_out/ab_${TAG}_p${P}_$pass.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/ab_${TAG}_p${P}_$pass.json'));r=d['roofline']
ss={(x['numel'],x['publish'],x['learners_per_launch']):x['frac'] for x in r['size_sweep']}
print('pass $pass policy $P value',d['value'],'frac',r['frac'],'inloop',r['in_loop']['avg_launch_us'],'wt',d['reference_loop']['value'],
  'res1',ss[(11173962,'resident',1)],'wt1',ss[(11173962,'write-through',1)],'wt2',ss[(11173962,'write-through',2)],
  'res1_100m',ss[(100000000,'resident',1)],'res1_7b',ss[(7000000000,'resident',1)],'rs',[x['value'] for x in d['round_sweep']])
"
  done
done
