#!/bin/bash
# HEAD verification (tools/gpu_r3_head.sh), then training tests on ab/lib_$NEW.so and a C4 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
bash tools/gpu_r3_head.sh || exit 1
cp ab/lib_$NEW.so no-node-comparison_amd/libnonode.so
TESTS="tests/test_gpu_train.py tests/test_gpu_train_segno.py tests/test_gpu_dp.py" timeout -k 10 400 bash tools/gpu_tests.sh && LIBS="base $NEW" bash tools/ab_train.sh
