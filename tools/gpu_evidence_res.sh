#!/bin/bash
# Evidence of the resident form (the bench's default publish form) for profiles/:
#  1. PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md §HBM) of
#     the cold resident averaging kernels: the batched dispatch of two learners (N=1's kernel) and
#     the single kernel (N>1's);
#  2. rocprofv3 --kernel-trace --stats of the driver's bench command (CPU baseline skipped: it
#     launches no kernel), split per grid and per run of consecutive dispatches;
#  3. the driver's bench command itself with the traffic of step 1.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_evidence_res.sh <tag>
set -o pipefail
TAG=${1:-res}
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in 2 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_res_${c}_x$L -o p -- \
        python3 tools/cold_sweep.py --publish resident --learners $L > gpurun_out/pmc_res_${c}_x$L.log 2>&1 \
        || { echo "$c pass x$L failed"; tail gpurun_out/pmc_res_${c}_x$L.log; exit 1; }
  done
  k="k_lerp<dpwa::OpsF32, 2, true, 64, 8, true>"; suf=""
  [ $L -gt 1 ] && { k="k_lerp_batch<dpwa::OpsF32, true, 8, true>"; suf="_x$L"; }
  python3 tools/pmc_traffic.py gpurun_out/pmc_res_FETCH_SIZE_x$L gpurun_out/pmc_res_WRITE_SIZE_x$L --kernel "$k" \
      --publish resident --learners $L --basis cold --out gpurun_out/traffic_${TAG}_resident$suf.json || exit 1
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/bench_rocprof_$TAG.json 2> gpurun_out/bench_rocprof_$TAG.err || { echo "rocprof bench failed"; tail gpurun_out/bench_rocprof_$TAG.err; exit 1; }
python3 tools/trace_stats.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_per_size.csv && \
  python3 tools/trace_stats.py --runs gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_runs.csv || exit 1
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 --traffic gpurun_out/traffic_${TAG}_resident_x2.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));r=d['roofline'];print('value',d['value'],'frac',r['frac'],r['avg_launch_us'],'traffic',r['traffic'],'inloop',r['in_loop']['avg_launch_us'],'sec',d.get('secondary_publish',{}).get('value'),'parity',{k:v for k,v in d.get('parity',{}).items() if k!='workload'})"
echo done
