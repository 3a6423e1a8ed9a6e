#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench. Each GPU step has its own time limit; a
# fault / abort / timeout (anything but pass=0 or test-failure=1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "fatal rc=$1 in $2"; exit "$1"; fi; }
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; stop_if_fatal $rc bench
exit 0
