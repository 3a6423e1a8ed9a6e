#!/bin/bash
# device assembly of the library (same flags as build()): bash tools/isa.sh <out.s> [-DFLAG=VAL ...]
cd "$(dirname "$0")/.."
out=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Wno-unused-value -mllvm -amdgpu-mfma-vgpr-form=1 ${SCHED--mllvm -amdgpu-sched-strategy=iterative-ilp} -I include "$@" --cuda-device-only -S -o "$out" no-node-comparison_amd/csrc/nonode.hip
