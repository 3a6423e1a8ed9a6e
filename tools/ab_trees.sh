#!/bin/bash
# Same-box A/B of two whole source trees (python + library), e.g. a previous commit checked out under
# ab/head (bench.py, the package with its built libnonode.so, oracle/, profiles/pmc_traffic.json):
#   ARMS="head:ab/head/bench.py new:bench.py newfe:bench.py@--optimizer foreach" WLS="egno_train:20:3" REPS=2 \
#     bash tools/ab_trees.sh
# prints step ms per arm and workload, alternating the arms REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/ab_trees}
mkdir -p "$O"
for rep in $(seq ${REPS:-2}); do
  for arm in ${ARMS}; do
    name=${arm%%:*}; rest=${arm#*:}; script=${rest%%@*}; extra=""; [ "$rest" != "$script" ] && extra=${rest#*@}
    line="$name"
    for spec in ${WLS:-egno_train:20:3}; do
      IFS=: read -r wl st wu <<< "$spec"
      f=$O/${name}_${wl}_$rep.json
      timeout -k 10 240 python3 $script --workload $wl --steps $st --warmup $wu --no-cpu-baseline ${extra//+/ } > $f 2> ${f%.json}.err \
        || { echo "fail $name $wl"; tail -3 ${f%.json}.err; exit 1; }
      line="$line $wl=$(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step'], 4))" $f)"
    done
    echo "$line"
  done
done
