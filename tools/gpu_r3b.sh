#!/bin/bash
# round-3 session B: same-box A/B of ab/lib_base.so (round-2 HEAD) and ab/lib_new.so over C2 / C3 /
# C4 (alternating, twice), then C4 at its real global batch (4096) on one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_r3b.log; [ $rc -gt 1 ] && exit $rc
fi
for n in ${LIBS:-base new base new}; do
  line="$n"
  for spec in egno:20:3 segno:20:3 egno_train:6:2; do
    IFS=: read -r wl st wu <<< "$spec"
    NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 200 python3 bench.py --workload $wl --steps $st --warmup $wu --no-cpu-baseline > gpurun_out/ab_${n}_$wl.json 2>/dev/null || { echo "fail $n $wl"; exit 1; }
    line="$line $wl=$(python3 -c "import json; d=json.load(open('gpurun_out/ab_${n}_$wl.json')); r=d.get('roofline') or {}; print(round(d['ms_per_step'], 4), round((r.get('avg_launch_ms') or 0)*1e3, 1))")"
  done
  echo "$line"
done
if [ "${C4_4096:-1}" = "1" ]; then
  timeout -k 10 400 python3 -u bench.py --workload egno_train --global-batch 4096 --gpus 1 --steps 6 --warmup 2 > gpurun_out/bench_egno_train_4096.json 2> gpurun_out/bench_egno_train_4096.err
  echo "c4 4096 rc=$?"; cut -c1-300 gpurun_out/bench_egno_train_4096.json; tail -2 gpurun_out/bench_egno_train_4096.err
fi
