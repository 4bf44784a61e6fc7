#!/bin/bash
# Round-6 evidence script: one parameterised GPU session (same steps as gpu_r05.sh, plus "line" after a bench).
#   tools/gpu_r06.sh <tag> <steps...>
# steps: smoke | tests:<pytest-args> | bench[:<bench args>] | rocprof[:<bench args>] | pmc:<cold_sweep args>
#        | marker[:<bench args>]  (DPWA_ROCTX=1 under rocprofv3 --marker-trace --kernel-trace)
#        | markerpy:<repo script + args>  (the same for a script, then tools/marker_gaps.py)
#        | rehearse:<N>[ <bench args>]  (the N>1 line self-launched on one GPU over gloo)
#        | py:<script + args>
# e.g. gpurun --timeout 1200 -- bash tools/gpu_r06.sh r05b smoke "tests:-m gpu tests" "bench:--steps 20 --warmup 5"
# Every step runs under its own timeout; the script stops at the first failing step.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i+1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "[gpu_r06 $tag] step $i: $step" >&2
  case $kind in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke failed" >&2; tail -30 "$out/smoke.log" >&2; exit 1; } ;;
    tests)
      timeout -k 10 1100 python -u -m pytest -x -v --timeout 280 --timeout-method thread $arg > "$out/pytest_$i.log" 2>&1 || { echo "tests failed" >&2; tail -60 "$out/pytest_$i.log" >&2; exit 1; } ;;
    ubsantests)   # the suite through build_san/libdpwa_hip.so (tools/ubsan_build.sh; take ./build_san out of .gpurunignore first)
      DPWA_HIP_LIB=$PWD/build_san/libdpwa_hip.so timeout -k 10 1100 python -u -m pytest -x -v --timeout 280 --timeout-method thread $arg > "$out/pytest_ubsan_$i.log" 2>&1 || { echo "ubsan tests failed" >&2; tail -60 "$out/pytest_ubsan_$i.log" >&2; exit 1; } ;;
    bench)
      DPWA_BENCH_DETAIL=$out/bench_${i}_detail.json timeout -k 10 900 python -u bench.py $arg > "$out/bench_$i.json" 2> "$out/bench_$i.err" || { echo "bench failed" >&2; tail -40 "$out/bench_$i.err" >&2; exit 1; }
      python3 tools/check_line.py "$out/bench_$i.json" >&2 || exit 1 ;;
    rocprof)
      (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/rocprof_$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $arg > "$GRAFT_REPO_ROOT/$out/rocprof_bench_$i.json" 2> "$GRAFT_REPO_ROOT/$out/rocprof_bench_$i.err") || { echo "rocprof failed" >&2; tail -40 "$out/rocprof_bench_$i.err" >&2; exit 1; } ;;
    marker)
      (cd /tmp && DPWA_ROCTX=1 timeout -k 10 900 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/marker_$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $arg > "$GRAFT_REPO_ROOT/$out/marker_bench_$i.json" 2> "$GRAFT_REPO_ROOT/$out/marker_bench_$i.err") || { echo "marker failed" >&2; tail -40 "$out/marker_bench_$i.err" >&2; exit 1; } ;;
    markerpy)
      (cd /tmp && DPWA_ROCTX=1 timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/markerpy_$i" -o run -- python3 $GRAFT_REPO_ROOT/$arg > "$GRAFT_REPO_ROOT/$out/markerpy_$i.log" 2>&1) || { echo "markerpy failed" >&2; tail -40 "$out/markerpy_$i.log" >&2; exit 1; }
      python3 tools/marker_gaps.py "$out/markerpy_$i" > "$out/markerpy_${i}_gaps.json" || exit 1 ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/pmc_${i}_$ctr" -o run -- python3 "$GRAFT_REPO_ROOT/tools/cold_sweep.py" $arg > "$GRAFT_REPO_ROOT/$out/pmc_${i}_$ctr.log" 2>&1) || { echo "pmc $ctr failed" >&2; tail -20 "$out/pmc_${i}_$ctr.log" >&2; exit 1; }
      done ;;
    rehearse)
      n=${arg%% *}; rest=${arg#"$n"}
      DPWA_BENCH_DETAIL=$out/rehearse_${i}_n${n}_detail.json timeout -k 10 900 python -u bench.py --gpus $n --dist-backend gloo --steps 20 --warmup 5 \
          --dist-sweep-max-numel 100000000 $rest > "$out/rehearse_${i}_n$n.json" 2> "$out/rehearse_${i}_n$n.err" \
          || { echo "rehearsal n=$n failed" >&2; tail -40 "$out/rehearse_${i}_n$n.err" >&2; exit 1; }
      python3 tools/check_line.py "$out/rehearse_${i}_n$n.json" >&2 || exit 1 ;;
    py)
      timeout -k 10 600 python -u $arg > "$out/py_$i.log" 2>&1 || { echo "py failed" >&2; tail -40 "$out/py_$i.log" >&2; exit 1; } ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "[gpu_r06 $tag] done" >&2
