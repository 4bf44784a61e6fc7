#!/bin/bash
# pair dispatch vs heap fragmentation and contiguous allocation (tools/pair_combo.hip)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pair_combo2.log
for args in "0 0" "64 0" "64 1" "4 0" "4 1" "0 1" "64 0"; do
  timeout -k 10 120 tools/pair_combo 11173962 4 400 $args > gpurun_out/pc.tmp 2>&1 || { cat gpurun_out/pc.tmp; exit 1; }
  cat gpurun_out/pc.tmp >> gpurun_out/pair_combo2.log
done
grep "mean over" gpurun_out/pair_combo2.log
