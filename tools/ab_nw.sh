#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for nw in 8 12; do
  NONODE_NW=$nw timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/nw_$nw.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/nw_$nw.json')); print('NW=$nw value=%.0f layer=%.1f us tconv=%.1f us' % (d['value'], d['roofline']['avg_launch_ms']*1e3, d['roofline']['tconv_avg_launch_ms']*1e3))"
done
