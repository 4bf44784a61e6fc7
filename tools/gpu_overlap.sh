set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gossip.py -m gpu -v --timeout 200 --timeout-method thread -k "prefetch" > gpurun_out/pytest_prefetch.log 2>&1; rc=$?; tail -6 gpurun_out/pytest_prefetch.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/overlap_g -o ov_%pid% -- \
    python3 tools/overlap_trace.py --batch 128 --steps 30 > gpurun_out/overlap_g.json 2> gpurun_out/overlap_g.err \
    || { echo "overlap trace failed"; tail -30 gpurun_out/overlap_g.err; exit 1; }
cat gpurun_out/overlap_g.json
python3 tools/overlap_trace.py --analyze gpurun_out/overlap_g
timeout -k 10 300 python3 tools/overlap_trace.py --batch 128 --steps 60 > gpurun_out/overlap_g_noprof_b128.json && cat gpurun_out/overlap_g_noprof_b128.json
timeout -k 10 300 python3 tools/overlap_trace.py --batch 8 --steps 60 > gpurun_out/overlap_g_noprof_b8.json && cat gpurun_out/overlap_g_noprof_b8.json
