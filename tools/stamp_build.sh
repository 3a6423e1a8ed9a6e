#!/bin/bash
# Diagnostic build with in-kernel s_memtime section stamps -> no-node-comparison_amd/libnonode_stamp.so
cd "$(dirname "$0")/.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize -Wno-unused-value -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=iterative-ilp -I include -DNONODE_STAMP=1 \
  -o no-node-comparison_amd/libnonode_stamp.so no-node-comparison_amd/csrc/nonode.hip
