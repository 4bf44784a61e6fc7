#!/bin/bash
# A pytest selection on the GPU.  Usage: gpurun -- bash tools/gpu_tests.sh <tag> "<selection>"
set -o pipefail
TAG=${1:-sel}; SEL=${2:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $SEL \
    > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -12; tail -3 gpurun_out/pytest_$TAG.log
exit $rc
