#!/bin/bash
# One-GPU rehearsal of the N>1 round sweep over the north_star sizes (gloo; the ranks share the
# GPU): N=2 self-launched with every size up to 7B bf16 (two ranks' learners fit in 288 GB),
# then the driver's launch line at N=8 with the sweep capped at 100M.  Each prints one line.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_rehearse_sweep.sh <tag>
set -o pipefail
TAG=${1:-sweep}
mkdir -p gpurun_out
export TMPDIR=/tmp
show() {
  python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['pull_choice']['chosen'],[(r['numel'],r.get('value',r.get('error'))) for r in d.get('round_sweep',[])])"
}
t0=$(date +%s)
timeout -k 10 900 python3 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo \
    > gpurun_out/sweep_${TAG}_n2.json 2> gpurun_out/sweep_${TAG}_n2.err
rc=$?
echo "N=2 rc=$rc $(( $(date +%s) - t0 ))s"
show gpurun_out/sweep_${TAG}_n2.json || exit 1
[ $rc -ne 0 ] && exit 1
t0=$(date +%s)
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29508 bench.py --gpus 8 --steps 20 --warmup 5 --dist-backend gloo \
    --dist-sweep-max-numel 100000000 > gpurun_out/sweep_${TAG}_n8.json 2> gpurun_out/sweep_${TAG}_n8.err
rc=$?
echo "N=8 rc=$rc $(( $(date +%s) - t0 ))s"
show gpurun_out/sweep_${TAG}_n8.json || exit 1
exit $rc
