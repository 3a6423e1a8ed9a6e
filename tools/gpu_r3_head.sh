#!/bin/bash
# GPU tests + smoke + C2 / C4 bench lines at HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3head
mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
NONODE_PARITY_REPORT=$O/parity_report.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke fail; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_egno.json 2> $O/bench_egno.err || { echo "bench c2 fail"; tail -5 $O/bench_egno.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload egno_train --steps 10 > $O/bench_egno_train.json 2> $O/bench_egno_train.err || { echo "bench c4 fail"; tail -5 $O/bench_egno_train.err; exit 1; }
for n in egno egno_train; do python3 -c "import json; d=json.load(open('$O/bench_$n.json')); r=d.get('roofline') or {}; print('$n', round(d['value']), 'ms', round(d['ms_per_step'],4), 'frac', r.get('frac'), 'avg', r.get('avg_launch_ms'), r.get('pass_ms'))"; done
