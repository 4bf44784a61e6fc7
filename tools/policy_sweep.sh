#!/bin/bash
# Cache-policy sweep of the averaging kernel inside the full gossip round (DPWA_LERP_POLICY
# 0-3, see LerpPolicy in kernels.hip), interleaved and repeated so run-to-run drift averages
# out.  Usage: gpurun --timeout 900 -- bash tools/policy_sweep.sh [numel] [repeats]
set -o pipefail
mkdir -p gpurun_out/policy
export TMPDIR=/tmp
N=${1:-11173962}
R=${2:-3}
V="--no-cpu-baseline --no-sweep --compute-us 0 --no-write-through --steps 200 --warmup 20 --numel $N"
for rep in $(seq 1 $R); do
  for p in 0 1 2 3; do
    DPWA_LERP_POLICY=$p timeout -k 10 120 python bench.py $V > gpurun_out/policy/p${p}_r${rep}_$N.json \
        2>> gpurun_out/policy/err.log || { echo "bench failed"; tail gpurun_out/policy/err.log; exit 1; }
    python - "$p" "gpurun_out/policy/p${p}_r${rep}_$N.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print("policy %s  value %8.1f GB/s  step %.4f ms  lerp live %.2f us (%.3f)  cold %.2f us (%.3f)" % (
    sys.argv[1], d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"],
    r["cold_cache"]["avg_launch_us"], r["cold_cache"]["frac"]), flush=True)
PY
  done
done
