#!/bin/bash
# Workgroup-size sweep of the averaging and publish kernels inside the full gossip round
# (bench.py, two co-resident learners), via the DPWA_LERP_BLOCK / DPWA_PUBLISH_BLOCK
# overrides.  Usage: gpurun --timeout 900 -- bash tools/block_sweep.sh [numel] [dtype]
set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
N=${1:-11173962}
DT=${2:-f32}
V="--no-cpu-baseline --no-sweep --compute-us 0 --no-write-through --steps 200 --warmup 20 --numel $N --dtype $DT"
for lb in 64 128 256 512; do
  for pb in 64 128 256; do
    DPWA_LERP_BLOCK=$lb DPWA_PUBLISH_BLOCK=$pb timeout -k 10 120 python bench.py $V \
        > gpurun_out/sweep/l${lb}_p${pb}_$N.json 2>> gpurun_out/sweep/err.log || { echo "bench failed"; tail gpurun_out/sweep/err.log; exit 1; }
    python - "$lb" "$pb" "gpurun_out/sweep/l${lb}_p${pb}_$N.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r = d["roofline"]
print("lerp %3s publish %3s  value %8.1f GB/s  step %.4f ms  lerp live %.2f us (%.3f)  cold %.2f us (%.3f)" % (
    sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"],
    r["cold_cache"]["avg_launch_us"], r["cold_cache"]["frac"]), flush=True)
PY
  done
done
