#!/bin/bash
# LDS-DMA / waves-per-workgroup A/B of the write-through kernel with the variant order controlled
# (round 6): order A and order B interleaved, 2 passes each at 11.17M, order A at 100M.
# Usage: gpurun --timeout 600 -- bash tools/tune_order_ab.sh   (after building tools/product_tune)
mkdir -p gpurun_out/r06f
A="product write-through;glds dual in place (nt, 2;glds dual in place (nt, 4;vgpr dual in place (nt, 2;glds dual in place (nt, 1"
B="glds dual in place (nt, 1;vgpr dual in place (nt, 2;glds dual in place (nt, 4;glds dual in place (nt, 2;product write-through"
for p in 1 2; do
  TUNE_ONLY="$A" timeout -k 10 120 tools/product_tune 11173962 20 > gpurun_out/r06f/order_a_pass$p.log 2>&1 || exit 1
  TUNE_ONLY="$B" timeout -k 10 120 tools/product_tune 11173962 20 > gpurun_out/r06f/order_b_pass$p.log 2>&1 || exit 1
done
TUNE_ONLY="$A" timeout -k 10 200 tools/product_tune 100000000 10 > gpurun_out/r06f/order_a_100m.log 2>&1
