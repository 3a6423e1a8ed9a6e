#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ counters) of the
# default bench workload. Output under gpurun_out/prof_${TAG}/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${TAG:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
BARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BARGS > $OUT/trace_bench.json 2> $OUT/trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ "${LIST:-0}" = "1" ]; then timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true; fi
for ctr in ${PMCS:-FETCH_SIZE WRITE_SIZE}; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-events > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
