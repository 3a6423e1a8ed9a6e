#!/bin/bash
# A/B the layer-kernel wave configurations (NONODE_CFG) on the C2 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CFGS:-0 1 2}; do
  NONODE_CFG=$c timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/cfg_$c.json 2>gpurun_out/cfg_$c.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/cfg_$c.json')); print('cfg=$c value=%.0f layer=%.1f us' % (d['value'], d['roofline']['avg_launch_ms']*1e3))"
done
