#!/bin/bash
# One-GPU rehearsal of the driver's own multi-GPU launch line (external torch.distributed.run),
# over gloo (RCCL refuses several ranks per GPU): N=8, then N=2; each must print one line.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_rehearse_ext.sh <tag>
set -o pipefail
TAG=${1:-ext}
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in 8 2; do
  t0=$(date +%s)
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29500 + N)) bench.py --gpus $N --steps 20 --warmup 5 --dist-backend gloo \
      --dist-sweep-max-numel 100000000 \
      > gpurun_out/ext_${TAG}_n$N.json 2> gpurun_out/ext_${TAG}_n$N.err
  rc=$?
  echo "N=$N rc=$rc $(( $(date +%s) - t0 ))s stdout lines: $(wc -l < gpurun_out/ext_${TAG}_n$N.json)"
  python3 tools/check_line.py gpurun_out/ext_${TAG}_n$N.json || exit 1
  [ $rc -ne 0 ] && exit 1
done
exit 0
