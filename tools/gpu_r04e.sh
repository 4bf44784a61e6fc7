#!/bin/bash
# Round 4: mutual-pair read sharing (tools/pair_tune.hip) at 11.17M (twice) and 100M fp32.
set -o pipefail
TAG=${1:-r04e}
mkdir -p gpurun_out
for run in "11173962 12 11m" "100000000 4 100m" "11173962 12 11m_b"; do
  set -- $run
  timeout -k 10 240 tools/pair_tune $1 $2 > gpurun_out/pair_tune_${TAG}_$3.log 2>&1 || { cat gpurun_out/pair_tune_${TAG}_$3.log; exit 1; }
  cat gpurun_out/pair_tune_${TAG}_$3.log
done
