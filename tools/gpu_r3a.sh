#!/bin/bash
# round-3 session A: pack decode check, all GPU tests, C2/C3 bench, then the edge-backward AGPR-pin
# diagnostic build (ab/lib_pin.so, NONODE_BWD_PIN=1) against the training tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
timeout -k 10 200 python tools/debug_pack.py > gpurun_out/debug_pack.log 2>&1 || { echo "debug_pack rc=$?"; exit 1; }
WORKLOADS="egno segno" bash tools/gpu_session.sh || exit $?
if [ -f ab/lib_pin.so ]; then
  NONODE_LIB=ab/lib_pin.so timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pin_train.log 2>&1
  echo "pin variant train tests rc=$?"; tail -3 gpurun_out/pin_train.log
fi
