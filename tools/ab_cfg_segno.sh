#!/bin/bash
# NONODE_CFG (layer-kernel wave configuration) A/B on the C3 SEGNO and C2 EGNO workloads
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for wl in segno egno; do for cfg in 1 0 2; do
  NONODE_CFG=$cfg timeout -k 10 120 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/cfg_${wl}_$cfg.json 2>gpurun_out/cfg_${wl}_$cfg.err || { echo "fail $wl $cfg"; tail -3 gpurun_out/cfg_${wl}_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfg_${wl}_$cfg.json')); r=d.get('roofline') or {}; print('$wl cfg=$cfg ms=%.4f kernel=%.1f us' % (d['ms_per_step'], (r.get('avg_launch_ms') or 0)*1e3))"
done; done
