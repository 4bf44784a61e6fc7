#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/pair_layout 11173962 400 > gpurun_out/pair_layout_${1:-r04i}.log 2>&1; rc=$?; cat gpurun_out/pair_layout_${1:-r04i}.log; exit $rc
