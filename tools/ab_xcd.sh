#!/bin/bash
# GPU tests with the XCD-aware TimeConv / layer order, then C2 and C4 with NONODE_XCD=1 vs 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xcd_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/xcd_pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in 1 0; do
  NONODE_XCD=$v timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/xcd_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/xcd_$v.json')); r=d['roofline']; print('XCD=$v ms=%.4f layer=%.1f tconv=%.1f us' % (d['ms_per_step'], r['avg_launch_ms']*1e3, r['tconv_avg_launch_ms']*1e3))"
done; done
