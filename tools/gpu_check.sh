#!/bin/bash
# One GPU-box pass: GPU parity tests, the default bench line, the kernel variant sweep
# (cold and Infinity-Cache warm), and the rocprofv3 kernel summary of the bench command.
# Usage (from this container): gpurun --timeout 1200 -- bash tools/gpu_check.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest -m gpu failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
# the other north_star configs, full gossip rounds on one GPU (two co-resident learners)
V="--no-cpu-baseline --no-sweep --no-cold --compute-us 0 --steps 50 --warmup 10"
timeout -k 10 200 python bench.py $V --numel 100000000 --interpolation clock > gpurun_out/bench_100m_clock.json 2>> gpurun_out/bench.err &&
timeout -k 10 200 python bench.py $V --numel 1000000000 --dtype bf16 --interpolation loss --divergence-threshold 0.5 --loss-schedule decay \
    > gpurun_out/bench_1b_bf16_loss.json 2>> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py $V --numel 7000000000 --dtype bf16 --fetch-probability 0.7 \
    > gpurun_out/bench_7b_bf16_p07.json 2>> gpurun_out/bench.err || { echo "variant bench failed"; tail gpurun_out/bench.err; exit 1; }
if [ -x tools/lerp_tune ]; then
    timeout -k 10 120 ./tools/lerp_tune 11173962 10 > gpurun_out/tune_cold.log 2>&1 || exit 1
    timeout -k 10 120 ./tools/lerp_tune 11173962 10 1 > gpurun_out/tune_warm.log 2>&1 || exit 1
    timeout -k 10 200 ./tools/lerp_tune 100000000 6 > gpurun_out/tune_cold_100m.log 2>&1 || exit 1
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --no-cpu-baseline --no-sweep > gpurun_out/bench_rocprof.json 2> gpurun_out/bench_rocprof.err || { echo "rocprof run failed"; exit 1; }
cat gpurun_out/bench_rocprof.json
echo done
