#!/bin/bash
# A/B of library builds ab/lib_<name>.so over the C2 / C3 / f1 / C4 workloads: LIBS="a b" bash tools/ab_all.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for n in ${LIBS}; do
  line="$n"
  for spec in egno:20:3 segno:20:3 egno_rollout:5:1 egno_train:6:2; do
    IFS=: read -r wl st wu <<< "$spec"
    NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 200 python3 bench.py --workload $wl --steps $st --warmup $wu --no-cpu-baseline > gpurun_out/ab_${n}_$wl.json 2>/dev/null || { echo "fail $n $wl"; exit 1; }
    line="$line $wl=$(python3 -c "import json; print(round(json.load(open('gpurun_out/ab_${n}_$wl.json'))['ms_per_step'], 4))")"
  done
  echo "$line"
done
