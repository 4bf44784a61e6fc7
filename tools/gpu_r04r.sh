#!/bin/bash
# Round 4, fused pair kernel: the pair / batch / resident suites, then the evidence script (PMC,
# rocprofv3, the driver's bench command).
set -o pipefail
TAG=${1:-r04r}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pairs.py \
    tests/test_gpu_batch.py tests/test_gpu_resident.py > gpurun_out/pytest_pairs_$TAG.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/pytest_pairs_$TAG.log | head; tail -30 gpurun_out/pytest_pairs_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_pairs_$TAG.log
bash tools/gpu_evidence_r04.sh $TAG
