#!/bin/bash
# round-3 session C: GPU parity tests (all, or TESTS=...), then a same-box A/B of library builds
# (LIBS, ab/lib_<name>.so) over the workloads in WLS (name:steps:warmup)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
if [ "${TESTS:-tests}" != "none" ]; then
  NONODE_PARITY_REPORT=gpurun_out/parity_report.json timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -8; [ $rc -gt 1 ] && exit $rc
fi
for n in ${LIBS:-}; do
  line="$n"
  for spec in ${WLS:-egno:20:3 segno:20:3 segno_gravity:10:2}; do
    IFS=: read -r wl st wu <<< "$spec"
    NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 200 python3 bench.py --workload $wl --steps $st --warmup $wu --no-cpu-baseline > gpurun_out/ab_${n}_$wl.json 2>gpurun_out/ab_${n}_$wl.err || { echo "fail $n $wl"; tail -3 gpurun_out/ab_${n}_$wl.err; exit 1; }
    line="$line $wl=$(python3 -c "import json; d=json.load(open('gpurun_out/ab_${n}_$wl.json')); r=d.get('roofline') or {}; print(round(d['ms_per_step'], 4), round((r.get('avg_launch_ms') or 0)*1e3, 1))")"
  done
  echo "$line"
done
