#!/bin/bash
# The driver's N>1 bench path rehearsed on one GPU (gloo: RCCL refuses two ranks per GPU),
# plus the C4/C5 config variants.  Usage: gpurun --timeout 900 -- bash tools/gpu_rehearse.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --dist-backend gloo --dist-sweep-max-numel 100000000 --steps 40 --warmup 5 --compute-us 300 \
      > gpurun_out/rehearse_n$n.json 2> gpurun_out/rehearse_n$n.err || { echo "rehearsal n=$n failed"; tail -20 gpurun_out/rehearse_n$n.err; exit 1; }
  cat gpurun_out/rehearse_n$n.json
done
# six ranks on one GPU: with the default 4 hardware queues per process the card's queue
# slots are oversubscribed (24) and host-synchronised rounds stall ~20 ms; 2 per process fit
GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 6 --master-addr 127.0.0.1 \
    --master-port 29506 bench.py --gpus 6 --dist-backend gloo --dist-sweep-max-numel 100000000 --steps 40 --warmup 5 --compute-us 300 \
    > gpurun_out/rehearse_n6.json 2> gpurun_out/rehearse_n6.err || { echo "rehearsal n=6 failed"; tail -20 gpurun_out/rehearse_n6.err; exit 1; }
cat gpurun_out/rehearse_n6.json
# configs[3]'s size across two processes: 4 GB of slots per rank, shared as hipMemCreate fds
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --dist-backend gloo --dist-sweep-max-numel 100000000 --numel 1000000000 --dtype bf16 --interpolation loss \
    --divergence-threshold 0.5 --loss-schedule decay --steps 20 --warmup 3 --compute-us 0 \
    > gpurun_out/rehearse_n2_1b.json 2> gpurun_out/rehearse_n2_1b.err || { echo "rehearsal 1B failed"; tail -20 gpurun_out/rehearse_n2_1b.err; exit 1; }
tail -1 gpurun_out/rehearse_n2_1b.json
V="--no-cpu-baseline --no-sweep --no-cold --compute-us 0 --steps 50 --warmup 10"
timeout -k 10 200 python bench.py $V --numel 100000000 --interpolation clock > gpurun_out/bench_100m_clock.json 2> gpurun_out/variants.err || { echo "variant failed"; tail gpurun_out/variants.err; exit 1; }
timeout -k 10 200 python bench.py $V --numel 1000000000 --dtype bf16 --interpolation loss --divergence-threshold 0.5 \
    --loss-schedule decay > gpurun_out/bench_1b_bf16_loss_decay.json 2> gpurun_out/variants.err &&
timeout -k 10 300 python bench.py $V --numel 7000000000 --dtype bf16 --fetch-probability 0.7 \
    > gpurun_out/bench_7b_bf16_p07.json 2>> gpurun_out/variants.err || { echo "variant failed"; tail gpurun_out/variants.err; exit 1; }
echo done
