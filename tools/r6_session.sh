# round-6 GPU session: full GPU tests, smoke, then C2 bench lines at B = 512 (headline), 256, 128, 64
set -u
cd "${GRAFT_REPO_ROOT}"
O=${O:-gpurun_out/r6d}; mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  NONODE_PARITY_REPORT=$O/parity_report.json timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $O/pytest_gpu.log | tail -8
  [ $rc -gt 1 ] && exit $rc
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke fail; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
BENCHES=${BENCHES:-"egno:--steps 20|b256:--batch 256 --steps 30 --no-cpu-baseline|b128:--batch 128 --steps 40 --no-cpu-baseline|b64:--batch 64 --steps 50 --no-cpu-baseline"}
IFS='|' read -ra specs <<< "$BENCHES"
for spec in "${specs[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 400 python -u bench.py $args > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $name fail"; tail -3 $O/bench_$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$name.json')); r=d.get('roofline') or {}; h=d.get('host_overhead') or {}
print('$name', round(d['value']), round(d['ms_per_step'],4), 'kern', round((r.get('avg_launch_ms') or 0)*1e3,1), 'tconv', round((r.get('tconv_avg_launch_ms') or 0)*1e3,1), 'frac', r.get('frac') and round(r['frac'],4), 'cpu', (d.get('cpu_baseline') or {}).get('value'), (d.get('cpu_baseline') or {}).get('calls'), 'host', h.get('enqueue_ms_median'))"
done
