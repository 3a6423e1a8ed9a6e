#!/bin/bash
# Time the layer kernel with phases skipped (NONODE_DEBUG bitmask; outputs are wrong, timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 0 1 2 4 3 5 6 7; do
  NONODE_DEBUG=$d timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ablate_$d.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ablate_$d.json')); print('debug=$d layer_ms=%.1f us tconv=%.1f us' % (d['roofline']['avg_launch_ms']*1e3, d['roofline']['tconv_avg_launch_ms']*1e3))"
done
