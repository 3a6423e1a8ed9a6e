#!/bin/bash
# Round profile set: for each workload in WORKLOADS a rocprofv3 --kernel-trace --stats run of the bench
# (its JSON line kept beside the trace), then separate FETCH_SIZE / WRITE_SIZE passes for the workloads
# in PMC_WORKLOADS. Output under gpurun_out/prof_${TAG}_<workload>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${TAG:-r02}
for wl in ${WORKLOADS:-egno segno segno_gravity egno_train egno_rollout}; do
  OUT=gpurun_out/prof_${TAG}_$wl
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
  rc=$?; echo "trace $wl rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/trace.err; exit $rc; }
done
for wl in ${PMC_WORKLOADS:-egno segno}; do
  OUT=gpurun_out/prof_${TAG}_$wl
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o run -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-events > /dev/null 2> $OUT/pmc_$ctr.err
    rc=$?; echo "pmc $wl $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/pmc_$ctr.err; exit $rc; }
  done
done
exit 0
