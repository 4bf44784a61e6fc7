#!/bin/bash
# Round 4: product kernels beside bare streams in one harness (tools/product_tune.hip), product
# policy 8 and sc0+sc1 (2), twice each.  Usage: gpurun -- bash tools/gpu_r04d.sh <tag>
set -o pipefail
TAG=${1:-r04d}
mkdir -p gpurun_out
for i in 1 2; do
  for P in 8 2; do
    DPWA_LERP_POLICY=$P timeout -k 10 180 tools/product_tune 11173962 12 > gpurun_out/product_tune_${TAG}_p${P}_$i.log 2>&1 || exit 1
    cat gpurun_out/product_tune_${TAG}_p${P}_$i.log
  done
done
