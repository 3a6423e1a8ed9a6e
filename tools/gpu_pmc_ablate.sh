#!/bin/bash
# PMC counters of the layer kernel with NONODE_DEBUG ablation (default 6: phase B only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-abl}
mkdir -p $OUT
export NONODE_DEBUG=${DBG:-6}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit $?
for ctr in ${PMCS}; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-events > /dev/null 2>&1 || exit $?
done
