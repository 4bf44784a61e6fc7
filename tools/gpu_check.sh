#!/bin/bash
# GPU check pass: the -m gpu suite, then the default bench line.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_check.sh <tag> [pytest selection...]
set -o pipefail
TAG=${1:-check}
shift
SEL=${@:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest $SEL -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu_$TAG.log | grep -E "FAIL|ERROR|passed|failed|Error" | tail -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 1; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
