#!/bin/bash
# The streaming-shape tuner at 11.17M and 100M fp32 (out-of-place resident shapes included), then
# the end-of-round check (smoke, the -m gpu suite, the default bench line).
# Usage: gpurun --timeout 1200 -- bash tools/gpu_final_st.sh <tag>
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 150 ./tools/stream_tune 11173962 10 > gpurun_out/st_${TAG}_11m.log 2>&1 || { echo "stream_tune 11m failed"; tail gpurun_out/st_${TAG}_11m.log; exit 1; }
timeout -k 10 200 ./tools/stream_tune 100000000 5 > gpurun_out/st_${TAG}_100m.log 2>&1 || { echo "stream_tune 100m failed"; tail gpurun_out/st_${TAG}_100m.log; exit 1; }
grep -E "oop|avg  64x1 \(|dual 64x1 \(|copy" gpurun_out/st_${TAG}_11m.log gpurun_out/st_${TAG}_100m.log
bash tools/gpu_final_r03.sh $TAG
