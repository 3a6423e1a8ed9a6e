#!/bin/bash
# round-3 close-out, part 1: GPU tests (parity report), smoke, one plain bench line per workload
# (C2 headline, C3, C5, C4 at 512 and at the 4096 global batch, f1 rollout, f3 simulator)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3final
mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
NONODE_PARITY_REPORT=$O/parity_report.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke fail; tail -5 $O/smoke.log; exit 1; }
cat $O/smoke.log | tail -1
for spec in "egno::" "segno::--steps 20" "segno_gravity::--steps 10" "egno_train::--steps 10" "egno_train_4096::--workload egno_train --global-batch 4096 --steps 5 --warmup 2" "egno_rollout::--steps 10" "sim_charged::--steps 3 --warmup 1"; do
  name=${spec%%::*}; args=${spec#*::}
  case $name in egno|egno_train_4096) wl="";; *) wl="--workload $name";; esac
  timeout -k 10 300 python -u bench.py $wl $args > $O/bench_$name.json 2> $O/bench_$name.err
  rc=$?; echo "bench $name rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/bench_$name.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/bench_$name.json')); r=d.get('roofline') or {}; print('$name', round(d['value']), d['unit'], 'ms', round(d['ms_per_step'],4), 'frac', r.get('frac'))"
done
echo done
