#!/bin/bash
# Every bench workload once (C3, C5, C4, row f1 rollout, row f3 simulator) plus a rocprofv3
# kernel-trace --stats pass of each. Output: gpurun_out/wl_${TAG}/<workload>.json, <workload>_stats/.
# Each GPU step has its own time limit; a nonzero status ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${TAG:-r01}
OUT=gpurun_out/wl_${TAG}
mkdir -p $OUT
for spec in ${WORKLOADS:-"segno:20:3" "segno_gravity:10:2" "egno_train:10:3" "egno_rollout:10:2" "sim_charged:3:1"}; do
  IFS=: read -r wl steps warm <<< "$spec"
  echo "== $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps $steps --warmup $warm > $OUT/$wl.json 2> $OUT/$wl.err
  rc=$?; echo "bench $wl rc=$rc"; cat $OUT/$wl.json; [ $rc -ne 0 ] && { tail -5 $OUT/$wl.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${wl}_stats -o run -- python3 bench.py --workload $wl --steps $steps --warmup $warm --no-cpu-baseline --no-kernel-events > $OUT/${wl}_prof.json 2> $OUT/${wl}_prof.err
  rc=$?; echo "rocprof $wl rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/${wl}_prof.err; exit $rc; }
done
exit 0
