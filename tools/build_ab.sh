#!/bin/bash
# build an A/B variant: bash tools/build_ab.sh <name> -DFLAG=VAL ...
cd "$(dirname "$0")/.."
n=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize -Wno-unused-value -mllvm -amdgpu-mfma-vgpr-form=1 ${SCHED--mllvm -amdgpu-sched-strategy=iterative-ilp} -I include "$@" -o ab/lib_$n.so no-node-comparison_amd/csrc/nonode.hip
