set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02x.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_r02x.log; exit 1; }
bash tools/gpu_check.sh r02x || exit 1
GPU_MAX_HW_QUEUES=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --dist-backend gloo --steps 40 --warmup 5 --compute-us 300 > gpurun_out/rehearse_x_n8.json 2> gpurun_out/rehearse_x_n8.err || { echo n8 failed; tail -20 gpurun_out/rehearse_x_n8.err; exit 1; }
tail -c 400 gpurun_out/rehearse_x_n8.json
