#!/bin/bash
# End-of-round check as the driver runs it: smoke(), the -m gpu suite, the default bench line.
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
bash tools/gpu_step.sh $TAG tests "--steps 20 --warmup 5" || exit 1
