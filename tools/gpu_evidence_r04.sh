#!/bin/bash
# Round 4 evidence for profiles/:
#  1. PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md §HBM) of the
#     four cold averaging kernels the line reports: resident batched (N=1 headline) and single (N>1),
#     write-through batched and single (the reference loop's form);
#  2. rocprofv3 --kernel-trace --stats of the driver's bench command (CPU baseline skipped: it launches
#     no kernel), split per grid size and per run of consecutive dispatches;
#  3. the driver's bench command itself (CPU baseline on), reading the traffic of step 1.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_evidence_r04.sh <tag>
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_launch.py \
    > gpurun_out/pytest_launch_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_launch_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_launch_$TAG.log
for fl in resident-pair:2 resident:1 write-through:2 write-through:1; do
  form=${fl%:*}; L=${fl#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${TAG}_${form}_${c}_x$L -o p -- \
        python3 tools/cold_sweep.py --publish $form --learners $L > gpurun_out/pmc_${TAG}_${form}_${c}_x$L.log 2>&1 \
        || { echo "$c pass $form x$L failed"; tail gpurun_out/pmc_${TAG}_${form}_${c}_x$L.log; exit 1; }
  done
  oop=$([ $form = write-through ] && echo false || echo true)
  k="k_lerp<dpwa::OpsF32, 2, true, 64, 8, $oop>"; suf=""
  [ $L -gt 1 ] && { k="k_lerp_batch<dpwa::OpsF32, true, 8, $oop>"; suf="_x$L"; }
  [ $form = resident-pair ] && k="k_lerp_pair<dpwa::OpsF32, 8>"
  python3 tools/pmc_traffic.py gpurun_out/pmc_${TAG}_${form}_FETCH_SIZE_x$L gpurun_out/pmc_${TAG}_${form}_WRITE_SIZE_x$L \
      --kernel "$k" --publish $form --learners $L --basis cold --out gpurun_out/traffic_${TAG}_$form$suf.json || exit 1
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/bench_rocprof_$TAG.json 2> gpurun_out/bench_rocprof_$TAG.err || { echo "rocprof bench failed"; tail gpurun_out/bench_rocprof_$TAG.err; exit 1; }
python3 tools/trace_stats.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_per_size.csv && \
  python3 tools/trace_stats.py --runs gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_runs.csv || exit 1
mkdir -p gpurun_out/traffic_$TAG && cp gpurun_out/traffic_${TAG}_*.json gpurun_out/traffic_$TAG/
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 --traffic gpurun_out/traffic_${TAG}_resident-pair_x2.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));r=d['roofline'];print('value',d['value'],'frac',r['frac'],r['avg_launch_us'],'traffic',r['traffic'],'inloop',r['in_loop']['avg_launch_us'],'parity',{k:v for k,v in d.get('parity',{}).items() if k!='workload'});print(json.dumps(d['reference_loop']))"
for f in gpurun_out/traffic_${TAG}_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d.get('hbm_bytes_per_launch'), d.get('ratio', d.get('traffic_over_algorithmic')))"; done
echo done
