#!/bin/bash
# Evidence pass for the profiles/ directory (run after the kernels change):
#  1. PMC HBM traffic of the averaging kernel, cold (tools/cold_sweep.py at configs[1]), both
#     publish forms, FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md §HBM);
#  2. rocprofv3 kernel trace of the cold sweep at every north_star size;
#  3. f1: the ResNet-18 trainer with gossip, 2 co-resident learners (step overhead), and the
#     2-process overlap trace (side-stream pull vs the training step's kernels);
#  4. the default bench line with that traffic, and its rocprofv3 kernel summary.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_evidence.sh <tag>
set -o pipefail
TAG=${1:-ev}
mkdir -p gpurun_out
export TMPDIR=/tmp
for form in full write-through; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f_$form -o f -- \
      python3 tools/cold_sweep.py --publish $form > gpurun_out/pmc_f_$form.log 2>&1 || { echo "FETCH pass $form failed"; tail gpurun_out/pmc_f_$form.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w_$form -o w -- \
      python3 tools/cold_sweep.py --publish $form > gpurun_out/pmc_w_$form.log 2>&1 || { echo "WRITE pass $form failed"; tail gpurun_out/pmc_w_$form.log; exit 1; }
  k="k_lerp<dpwa::OpsF32, 2, false,"; [ $form = write-through ] && k="k_lerp<dpwa::OpsF32, 2, true,"
  python3 tools/pmc_traffic.py gpurun_out/pmc_f_$form gpurun_out/pmc_w_$form --kernel "$k" --publish $form \
      --basis cold --out gpurun_out/traffic_${TAG}_$form.json || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cold_$TAG -o cold -- \
    python3 tools/cold_sweep.py --all > gpurun_out/cold_sweep_$TAG.jsonl 2> gpurun_out/cold_sweep_$TAG.err \
    || { echo "cold sweep failed"; tail gpurun_out/cold_sweep_$TAG.err; exit 1; }
python3 tools/trace_stats.py gpurun_out/cold_$TAG/cold_kernel_trace.csv > gpurun_out/cold_${TAG}_per_size.csv || exit 1
for b in 8 128; do
  timeout -k 10 300 python3 examples/resnet18_gossip.py --learners 2 --steps 60 --batch-size $b \
      > gpurun_out/resnet18_b$b.json 2> gpurun_out/resnet18_b$b.err || { echo "resnet b$b failed"; tail gpurun_out/resnet18_b$b.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/overlap_$TAG -o ov_%pid% -- \
    python3 tools/overlap_trace.py --batch 128 --steps 30 > gpurun_out/overlap_$TAG.json 2> gpurun_out/overlap_$TAG.err \
    || { echo "overlap trace failed"; tail -30 gpurun_out/overlap_$TAG.err; exit 1; }
python3 tools/overlap_trace.py --analyze gpurun_out/overlap_$TAG > gpurun_out/overlap_${TAG}_analysis.json || exit 1
cat gpurun_out/overlap_${TAG}_analysis.json
timeout -k 10 600 python3 bench.py --traffic gpurun_out/traffic_${TAG}_write-through.json > gpurun_out/bench_$TAG.json \
    2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --traffic gpurun_out/traffic_${TAG}_write-through.json \
    > gpurun_out/bench_rocprof_$TAG.json 2> gpurun_out/bench_rocprof_$TAG.err || { echo "rocprof bench failed"; exit 1; }
python3 tools/trace_stats.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_per_size.csv && python3 tools/trace_stats.py --runs gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_runs.csv || exit 1
echo done
