set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/stream_tune 11173962 12 > gpurun_out/tune_11m.log 2>&1 && cat gpurun_out/tune_11m.log &&
timeout -k 10 200 tools/stream_tune 100000000 6 > gpurun_out/tune_100m.log 2>&1 && cat gpurun_out/tune_100m.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/pytest_configs.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_configs.log; exit $rc
