#!/bin/bash
# A/B of the reuse guard's index arithmetic: the adapter's round (tools/adapter_rounds.py, guard on,
# and the resident learner with its window guard) through build_gold/libdpwa_hip.so (the library
# before the change, built from the parent commit) and dpwa_amd/libdpwa_hip.so, interleaved over
# three passes, then one rocprofv3 --kernel-trace --stats run of each for the guard kernels' times.
#   gpurun -- bash tools/guard_ab.sh <tag>
set -o pipefail
tag=${1:-guard_ab}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
new=$PWD/dpwa_amd/libdpwa_hip.so
old=$PWD/build_gold/libdpwa_hip.so
for pass in 1 2 3; do
  for which in old new; do
    lib=$old; [ $which = new ] && lib=$new
    for mode in "" "--resident"; do
      echo "[guard_ab] pass $pass $which $mode" >&2
      DPWA_HIP_LIB=$lib timeout -k 10 180 python -u tools/adapter_rounds.py --rounds 2000 --warmup 100 $mode \
        >> "$out/rounds_$which.log" 2>&1 || { echo "adapter_rounds failed" >&2; tail -20 "$out/rounds_$which.log" >&2; exit 1; }
    done
  done
done
for which in old new; do
  lib=$old; [ $which = new ] && lib=$new
  (cd /tmp && DPWA_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/$out/prof_$which" -o run -- python3 "$GRAFT_REPO_ROOT/tools/adapter_rounds.py" --rounds 1000 \
      > "$GRAFT_REPO_ROOT/$out/prof_$which.log" 2>&1) || { echo "rocprof $which failed" >&2; tail -20 "$out/prof_$which.log" >&2; exit 1; }
done
echo "[guard_ab $tag] done" >&2
