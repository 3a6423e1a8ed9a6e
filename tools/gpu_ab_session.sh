#!/bin/bash
# GPU tests, then an A/B of library builds (LIBS, ab/lib_<name>.so) on the workloads in WORKLOADS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
if [ "${TESTS:-1}" = "1" ]; then
  NONODE_PARITY_REPORT=gpurun_out/parity_report.json timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for wl in ${WORKLOADS:-egno}; do
for rep in 1 2; do
for n in ${LIBS}; do
  NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 150 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${wl}_$n.json 2>gpurun_out/ab_${wl}_$n.err || { echo "fail $wl $n"; tail -3 gpurun_out/ab_${wl}_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_${wl}_$n.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$wl $n value=%.0f ms=%.4f kernel=%.1f us' % (d['value'], d['ms_per_step'], (r.get('avg_launch_ms') or 0)*1e3))"
done
done
done
