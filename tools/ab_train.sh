#!/bin/bash
# A/B library builds on the C4 training bench: for each ab/lib_<name>.so print step time and the
# edge-backward pass times. Usage: LIBS="a b" bash tools/ab_train.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for n in ${LIBS}; do
  NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 180 python3 bench.py --workload egno_train --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abt_$n.json 2>gpurun_out/abt_$n.err || { echo "fail $n"; tail -3 gpurun_out/abt_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abt_$n.json')); r=d.get('roofline') or {}; print('$n ms=%.3f edge_bwd=%.1f us passes=%s fwd_layer=%.1f parity=%s' % (d['ms_per_step'], (r.get('avg_launch_ms') or 0)*1e3, [round(x*1e3,1) for x in r.get('pass_ms',[])], (r.get('forward_layer_avg_ms') or 0)*1e3, (d.get('parity') or {}).get('grad_maxnorm_rel_vs_f64_max')))"
done
done
