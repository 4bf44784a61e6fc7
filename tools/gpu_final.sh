#!/bin/bash
# End-of-round evidence pass: PMC HBM traffic of the averaging kernel (FETCH_SIZE and
# WRITE_SIZE in separate passes), then the default bench line carrying that traffic, then
# the rocprofv3 kernel summary of the same bench command.
# Usage: gpurun --timeout 900 -- bash tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --no-sweep --no-cold --compute-us 0 --no-write-through --steps 100 --warmup 10"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 $B \
    > gpurun_out/pmc_fetch.log 2>&1 || { echo "FETCH_SIZE pass failed"; tail gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python3 $B \
    > gpurun_out/pmc_write.log 2>&1 || { echo "WRITE_SIZE pass failed"; tail gpurun_out/pmc_write.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --out gpurun_out/traffic_$TAG.json || exit 1
timeout -k 10 300 python3 bench.py --traffic gpurun_out/traffic_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --no-sweep --traffic gpurun_out/traffic_$TAG.json \
    > gpurun_out/bench_rocprof_$TAG.json 2> gpurun_out/bench_rocprof_$TAG.err || { echo "rocprof run failed"; exit 1; }
echo done
