#!/bin/bash
# One-GPU rehearsal of the N>1 bench path as the driver would start it WITHOUT a launcher
# (bench.py --gpus N self-launches torch.distributed.run as a child), over gloo:
#   1. a clean run -> one line, rc 0
#   2. an injected failure at the END of lockstep/relay:32 on rank 1 -> the transport's isolation
#      turns it into parity false, the run still prints its line, rc 1
#   3. an injected failure at the START of it on rank 1 (the other ranks block in a collective)
#      -> the watchdog prints a partial line and the job ends with rc != 0 within the bound
# Usage: gpurun --timeout 1200 -- bash tools/gpu_rehearse_r03.sh <tag> <N>
set -o pipefail
TAG=${1:-r03}
N=${2:-4}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--gpus $N --dist-backend gloo --dist-sweep-max-numel 100000000 --steps 20 --warmup 5 --no-cpu-baseline --compute-us 0"
t0=$(date +%s)
timeout -k 10 500 python -u bench.py $B > gpurun_out/rh_${TAG}_clean.json 2> gpurun_out/rh_${TAG}_clean.err
echo "clean rc=$? $(( $(date +%s) - t0 ))s, stdout lines: $(wc -l < gpurun_out/rh_${TAG}_clean.json)"
python3 -c "import json;d=json.load(open('gpurun_out/rh_${TAG}_clean.json'));print(d['value'], d.get('pull_choice'), {k:v for k,v in d['parity'].items() if k!='workload'})"
[ "${3:-all}" = "clean" ] && exit 0
t0=$(date +%s)
DPWA_BENCH_INJECT="lockstep/relay:32@1:end" timeout -k 10 500 python -u bench.py $B --no-secondary \
    > gpurun_out/rh_${TAG}_inject_end.json 2> gpurun_out/rh_${TAG}_inject_end.err
echo "inject-end rc=$? $(( $(date +%s) - t0 ))s, stdout lines: $(wc -l < gpurun_out/rh_${TAG}_inject_end.json)"; python -c "import json;d=json.load(open('gpurun_out/rh_${TAG}_inject_end.json'));print(d.get('parity'), d.get('value'))"
t0=$(date +%s)
DPWA_BENCH_INJECT="lockstep/relay:32@1:start" timeout -k 10 400 python -u bench.py $B --no-secondary --phase-scale 0.25 \
    > gpurun_out/rh_${TAG}_inject_start.json 2> gpurun_out/rh_${TAG}_inject_start.err
echo "inject-start rc=$? $(( $(date +%s) - t0 ))s, stdout lines: $(wc -l < gpurun_out/rh_${TAG}_inject_start.json)"; cat gpurun_out/rh_${TAG}_inject_start.json
exit 0
