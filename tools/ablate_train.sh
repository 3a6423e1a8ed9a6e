#!/bin/bash
# Time the C4 training step with parts of edge_bwd PASS 1 skipped (NONODE_EBDBG bitmask; gradients
# are wrong, timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 4 8 16 32 64 127}; do
  NONODE_EBDBG=$d timeout -k 10 120 python3 bench.py --workload egno_train --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/abt_$d.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/abt_$d.json')); print('dbg=$d ms_per_step=%.2f' % d['ms_per_step'])"
done
