#!/bin/bash
# Kernel variant sweep (tools/lerp_tune.hip): 11.2M fp32 cold and Infinity-Cache warm, 100M fp32 cold.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/lerp_tune 11173962 10 > gpurun_out/t_11m_cold.log 2>&1 &&
timeout -k 10 120 ./tools/lerp_tune 11173962 10 1 > gpurun_out/t_11m_warm.log 2>&1 &&
timeout -k 10 200 ./tools/lerp_tune 100000000 6 > gpurun_out/t_100m_cold.log 2>&1
