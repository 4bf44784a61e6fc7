set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 tools/pair_diag.py > gpurun_out/pair_diag5.log 2>&1 && \
DPWA_CONTIG=1 timeout -k 10 200 python3 tools/pair_diag.py > gpurun_out/pair_diag5_contig.log 2>&1 && \
PAIR_DIAG_ROUNDS=300 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pd -o pd -- python3 tools/pair_diag.py > gpurun_out/pair_diag5_prof.log 2>&1
rc=$?
grep -v -i "warning\|amdgpu.ids" gpurun_out/pair_diag5.log gpurun_out/pair_diag5_contig.log
exit $rc
