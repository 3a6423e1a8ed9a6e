#!/bin/bash
# GPU tests only (optionally a subset: TESTS="tests/test_gpu_rollout.py"), one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -25 gpurun_out/pytest_gpu.log; exit $rc
