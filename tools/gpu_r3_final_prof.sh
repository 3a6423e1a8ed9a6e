#!/bin/bash
# round-3 close-out, part 2: rocprofv3 kernel stats of every workload and FETCH_SIZE / WRITE_SIZE
# passes of C2, C3 and C4 (tools/gpu_profile_all.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03 PMC_WORKLOADS="egno segno egno_train" bash tools/gpu_profile_all.sh
