#!/bin/bash
# rocprofv3 kernel stats of library variants ab/lib_<name>.so ($LIBS) on one workload ($WL, bench args $ARGS)
# under gpurun_out/abprof_<name>/; prints the average ns of the kernels matching $KPAT per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
for rep in $(seq ${REPS:-1}); do
  for n in $LIBS; do
    out=gpurun_out/abprof_${n}_$rep
    NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
      python3 bench.py --workload ${WL:-egno} --steps 10 --warmup 2 --no-cpu-baseline ${ARGS:-} > $out.json 2> $out.err \
      || { echo "fail $n"; tail -3 $out.err; exit 1; }
    python3 - "$out/run_kernel_stats.csv" "$n" "${KPAT:-tconv}" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[3] in r["Name"]]
print(sys.argv[2], "; ".join("%s %.1f us x%s" % (r["Name"][:60], float(r["AverageNs"]) / 1e3, r["Calls"]) for r in rows))
PY
  done
done
