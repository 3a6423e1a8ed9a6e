#!/bin/bash
# round-3 session E: GPU tests at HEAD (parity report), C2 bench, C4 at 512/GPU and at the C4
# global batch 4096 on one GPU (N=1 point of the strong-scaling curve), edge-backward stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
NONODE_PARITY_REPORT=$O/parity_report.json timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_egno.json 2> $O/bench_egno.err || { echo "bench c2 fail"; tail -5 $O/bench_egno.err; exit 1; }
cat $O/bench_egno.json
timeout -k 10 300 python -u bench.py --workload egno_train --steps 10 --warmup 3 > $O/bench_egno_train.json 2> $O/bench_egno_train.err || { echo "bench c4 fail"; tail -5 $O/bench_egno_train.err; exit 1; }
cat $O/bench_egno_train.json
timeout -k 10 400 python -u bench.py --workload egno_train --global-batch 4096 --steps 5 --warmup 2 > $O/bench_egno_train_4096.json 2> $O/bench_egno_train_4096.err || { echo "bench c4 4096 fail"; tail -5 $O/bench_egno_train_4096.err; exit 1; }
cat $O/bench_egno_train_4096.json
S=no-node-comparison_amd/libnonode_stamp.so
NONODE_LIB=$PWD/$S timeout -k 10 120 python3 tools/stamp_train.py > $O/stamp_train.txt 2>&1 || { echo "stamp fail"; tail -5 $O/stamp_train.txt; exit 1; }
cat $O/stamp_train.txt
echo done
