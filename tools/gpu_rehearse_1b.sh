#!/bin/bash
# configs[3] (1B bf16, loss interpolation, divergence threshold 0.5, decaying loss) through the
# driver's launch line at N ranks on one GPU (gloo): fd-shared hipMemCreate slots (1.5 GiB and
# up), the relay buffers, the board, every parity transport.  Usage: gpurun -- bash tools/gpu_rehearse_1b.sh <tag> <N>
set -o pipefail
TAG=${1:-1b}; N=${2:-8}
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus $N --steps 10 --warmup 3 --dist-backend gloo --dist-sweep-max-numel 100000000 --numel 1000000000 --dtype bf16 \
    --interpolation loss --divergence-threshold 0.5 --loss-schedule decay --no-cpu-baseline --no-sweep --no-cold \
    --compute-us 0 --no-secondary --trial-passes 1 --phase-scale 3 \
    > gpurun_out/r1b_${TAG}_n$N.json 2> gpurun_out/r1b_${TAG}_n$N.err
rc=$?
echo "N=$N rc=$rc $(( $(date +%s) - t0 ))s stdout lines: $(wc -l < gpurun_out/r1b_${TAG}_n$N.json)"
python3 -c "import json;d=json.load(open('gpurun_out/r1b_${TAG}_n$N.json'));print(d['value'],d.get('pull_choice'),{k:v for k,v in d['parity'].items() if k!='workload'}, d.get('pull_trials_gbs'))"
exit $rc
