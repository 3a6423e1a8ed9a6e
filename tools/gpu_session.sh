#!/bin/bash
# One GPU-box session: GPU tests (all, with the measured-parity report), then bench lines for the
# workloads in WORKLOADS (default: C2 C3 C4 C5 f1). Each GPU step has its own time limit; a fault /
# abort / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "fatal rc=$1 in $2"; exit "$1"; fi; }
if [ "${TESTS:-1}" = "1" ]; then
  NONODE_PARITY_REPORT=gpurun_out/parity_report.json timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3; stop_if_fatal $rc pytest
fi
for wl in ${WORKLOADS:-egno segno egno_train segno_gravity egno_rollout}; do
  timeout -k 10 400 python -u bench.py --workload $wl ${BENCH_ARGS:-} > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
  rc=$?; echo "bench $wl rc=$rc"; cut -c1-400 gpurun_out/bench_$wl.json; tail -2 gpurun_out/bench_$wl.err; stop_if_fatal $rc bench_$wl
done
exit 0
