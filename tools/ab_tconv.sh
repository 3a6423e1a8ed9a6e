#!/bin/bash
# A/B library builds on the C2 bench: step time, layer and tconv launch times per ab/lib_<name>.so.
# Usage: LIBS="a b" bash tools/ab_tconv.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for n in ${LIBS}; do
  NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$n.json 2>gpurun_out/ab_$n.err || { echo "fail $n"; tail -3 gpurun_out/ab_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); r=d.get('roofline') or {}; print('$n value=%.0f ms=%.4f layer=%.1f us tconv=%.1f us' % (d['value'], d['ms_per_step'], (r.get('avg_launch_ms') or 0)*1e3, (r.get('tconv_avg_launch_ms') or 0)*1e3))"
done
done
