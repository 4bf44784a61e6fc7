#!/bin/bash
# Full pass after a kernel change: the -m gpu suite, the evidence (PMC traffic, rocprofv3 of the
# bench command, the bench line) and BASELINE configs[2..4] + the f1 trainer.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
bash tools/gpu_step.sh $TAG tests none || exit 1
bash tools/gpu_evidence_r03.sh $TAG || exit 1
bash tools/gpu_configs_r03.sh $TAG || exit 1
echo round-pass-done
