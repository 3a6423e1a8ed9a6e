#!/bin/bash
# phase-B internals: 6 = B only; +8 no edge-feature loads; +16 SiLU->clamp; +32 no fp16 MFMAs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 6 14 22 38 62; do
  NONODE_DEBUG=$d timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ablb_$d.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ablb_$d.json')); print('debug=$d layer=%.1f us' % (d['roofline']['avg_launch_ms']*1e3))"
done
