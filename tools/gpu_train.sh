#!/bin/bash
# Training path on the GPU box: gradient parity tests, then the C4 step bench (+ optional rocprof).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest train rc=$rc"; tail -15 gpurun_out/pytest_train.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload egno_train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_train.json; [ $rc -ne 0 ] && exit $rc
if [ "${PROF:-0}" = "1" ]; then
  mkdir -p gpurun_out/prof_train
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train/trace -o run -- python3 bench.py --workload egno_train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_train/bench.json 2> gpurun_out/prof_train/err.txt
  echo "prof rc=$?"
fi
exit 0
