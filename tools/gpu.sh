#!/bin/bash
# One parametrised GPU-box session (replaces the per-session gpu_r*.sh scripts of rounds 1-3).
#   bash tools/gpu.sh STEP [STEP ...]      e.g.  gpurun -- 'bash tools/gpu.sh tests bench'
# Steps (each GPU command under its own time limit; the session stops at the first fault, abort,
# time-out or failed bench, and pytest failures (rc 1) stop it unless KEEP_GOING=1):
#   tests    pytest -m gpu over $TESTS (default tests/), measured-parity report in $O/parity_report.json
#   smoke    __graft_entry__.smoke()
#   bench    one plain bench line per spec in $BENCH ("name:bench args", default: the C2 headline)
#   ab       same-box A/B of library builds ab/lib_<name>.so ($LIBS) over $WLS (workload:steps:warmup),
#            alternating $REPS times; prints step ms and the workload's roofline-kernel launch us
#   profile  rocprofv3 --kernel-trace --stats of $WORKLOADS, then FETCH_SIZE / WRITE_SIZE passes (one
#            counter per run) of the $PMC specs ("name:bench args" separated by '|'), under
#            gpurun_out/prof_${TAG}_<name>/
#   stamps   in-kernel section stamps (libnonode_stamp.so, tools/stamp_build.sh) of $STAMPS scripts
# Output directory: $O (default gpurun_out/session).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/session}
mkdir -p "$O"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1

jget() {   # jget FILE EXPR: a value of a bench JSON line
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print($2)" "$1"
}

step_tests() {
  NONODE_PARITY_REPORT=$O/parity_report.json timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  local rc=$?
  echo "pytest gpu rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $O/pytest_gpu.log | tail -8
  if [ $rc -gt 1 ] || { [ $rc -eq 1 ] && [ "${KEEP_GOING:-0}" != "1" ]; }; then exit $rc; fi
}

step_smoke() {
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke fail"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
}

step_bench() {
  local spec name args
  while IFS= read -r spec; do
    [ -z "$spec" ] && continue
    name=${spec%%:*}; args=${spec#*:}
    timeout -k 10 400 python -u bench.py $args > $O/bench_$name.json 2> $O/bench_$name.err
    local rc=$?; [ $rc -ne 0 ] && { echo "bench $name rc=$rc"; tail -5 $O/bench_$name.err; exit $rc; }
    echo "bench $name: $(jget $O/bench_$name.json "round(d['value']), d['unit'], 'ms', round(d['ms_per_step'], 4), 'kernel_us', round((r.get('avg_launch_ms') or 0) * 1e3, 1), 'frac', r.get('frac') and round(r['frac'], 4)")"
  done <<< "${BENCH:-egno:}"
}

step_ab() {
  local rep n spec wl st wu line f
  for rep in $(seq ${REPS:-2}); do
    for n in ${LIBS}; do
      line="$n"
      for spec in ${WLS:-egno:20:3}; do
        IFS=: read -r wl st wu <<< "$spec"
        f=$O/ab_${n}_$wl.json
        NONODE_LIB=$PWD/ab/lib_$n.so timeout -k 10 240 python3 bench.py --workload $wl --steps $st --warmup $wu \
          --no-cpu-baseline ${AB_ARGS:-} > $f 2> $O/ab_${n}_$wl.err || { echo "fail $n $wl"; tail -3 $O/ab_${n}_$wl.err; exit 1; }
        line="$line $wl=$(jget $f "round(d['ms_per_step'], 4), round((r.get('avg_launch_ms') or 0) * 1e3, 1), [round(x * 1e3, 1) for x in r.get('pass_ms', [])]")"
      done
      echo "$line"
    done
  done
}

step_profile() {
  local wl OUT ctr
  for wl in ${WORKLOADS-egno}; do
    OUT=gpurun_out/prof_${TAG:-r04}_$wl
    mkdir -p $OUT
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py \
      --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
    local rc=$?; echo "trace $wl rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/trace.err; exit $rc; }
  done
  # PMC: "name:bench args" specs separated by '|', e.g. PMC="c5:--workload segno_gravity|c4_4096:--workload
  # egno_train --global-batch 4096"
  local spec name args
  while IFS= read -r -d '|' spec; do
    [ -z "$spec" ] && continue
    name=${spec%%:*}; args=${spec#*:}
    OUT=gpurun_out/prof_${TAG:-r04}_$name
    mkdir -p $OUT
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o run -- python3 bench.py \
        $args --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-events > /dev/null 2> $OUT/pmc_$ctr.err
      local rc=$?; echo "pmc $name $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/pmc_$ctr.err; exit $rc; }
    done
  done <<< "${PMC:-}|"
}

step_stamps() {
  local s
  for s in ${STAMPS:-stamp_run.py}; do
    NONODE_LIB=$PWD/no-node-comparison_amd/libnonode_stamp.so timeout -k 10 180 python3 tools/$s > $O/${s%.py}.txt 2>&1 \
      || { echo "stamps $s fail"; tail -5 $O/${s%.py}.txt; exit 1; }
    cat $O/${s%.py}.txt
  done
}

for s in "$@"; do
  echo "== $s"
  step_$s
done
echo done
