#!/bin/bash
# round-3 session D: C3 vs C2 layer-kernel diagnosis: section stamps (stamp build) and one SQ PMC
# pass per workload (wave cycles split into active / issue-stall / parked, MFMA busy, VALU count)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
S=no-node-comparison_amd/libnonode_stamp.so
NONODE_LIB=$PWD/$S timeout -k 10 120 python3 tools/stamp_run_segno.py > gpurun_out/r3d/stamp_c3.txt 2>&1 || { echo "stamp c3 fail"; tail -5 gpurun_out/r3d/stamp_c3.txt; exit 1; }
cat gpurun_out/r3d/stamp_c3.txt
NONODE_WAVES=4 NONODE_LIB=$PWD/$S timeout -k 10 120 python3 tools/stamp_run.py > gpurun_out/r3d/stamp_c2.txt 2>&1 || { echo "stamp c2 fail"; tail -5 gpurun_out/r3d/stamp_c2.txt; exit 1; }
cat gpurun_out/r3d/stamp_c2.txt
for wl in segno egno; do
  WL=$wl TAG=r3d_$wl bash tools/pmc_layer.sh > gpurun_out/r3d/pmc_$wl.txt 2>&1 || { echo "pmc $wl fail"; tail -5 gpurun_out/r3d/pmc_$wl.txt; exit 1; }
  cat gpurun_out/r3d/pmc_$wl.txt
done
echo done
