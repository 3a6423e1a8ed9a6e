#!/bin/bash
# Round-end evidence in one GPU call: GPU tests, then tools/gpu_profile_all.sh (rocprofv3
# kernel-trace --stats of every workload + FETCH_SIZE / WRITE_SIZE passes). Each step has its own
# time limit; a fatal status ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
NONODE_PARITY_REPORT=gpurun_out/parity_report.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_profile_all.sh
