#!/bin/bash
# row †g bench line: SEGNO training step at the C3 configuration
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3st
mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u bench.py --workload segno_train --steps 10 --warmup 2 > $O/bench_segno_train.json 2> $O/err.log
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/err.log; exit $rc; }
python3 -c "import json; d=json.load(open('$O/bench_segno_train.json')); r=d.get('roofline') or {}; print(round(d['value']), d['ms_per_step'], r.get('frac'), r.get('pass_ms'), d.get('parity'), (d.get('cpu_baseline') or {}).get('value'))"
