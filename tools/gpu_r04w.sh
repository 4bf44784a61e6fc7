#!/bin/bash
# Round 4: k_lerp_group (closed groups of co-resident resident learners): the pair / batch /
# resident / gossip suites and the full-size resident configs, then G = 3 and 4 gossip rounds with it
# on and off (tools/group_round.py).
set -o pipefail
TAG=${1:-r04w}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pairs.py \
    tests/test_gpu_batch.py tests/test_gpu_resident.py tests/test_gpu_gossip.py \
    "tests/test_gpu_configs.py::test_full_size_configs_resident" "tests/test_gpu_configs.py::test_configs0_resnet18_resident_training" \
    > gpurun_out/pytest_$TAG.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for pass in ${PASSES:-1 2}; do
  for f in 1 0; do
    DPWA_PAIR_FUSED=$f timeout -k 10 300 python3 -u tools/group_round.py > gpurun_out/group_${TAG}_f${f}_$pass.log 2>&1 \
      || { tail -20 gpurun_out/group_${TAG}_f${f}_$pass.log; exit 1; }
    grep "^G" gpurun_out/group_${TAG}_f${f}_$pass.log | sed "s/^/fused=$f pass $pass /"
  done
done
