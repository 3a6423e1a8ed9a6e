#!/bin/bash
# device assembly of one translation unit (same flags as build()): bash tools/isa.sh <out.s> [-DFLAG=VAL ...]
# UNIT=nonode_node.hip for the node backward's unit (built with the default machine scheduler)
cd "$(dirname "$0")/.."
out=$1; shift
unit=${UNIT:-nonode.hip}
if [ "$unit" = nonode.hip ]; then sched=${SCHED--mllvm -amdgpu-sched-strategy=iterative-ilp}; else sched=${SCHED-}; fi
vf="-mllvm -amdgpu-mfma-vgpr-form=1"; [ "$unit" = nonode_tconv.hip ] && vf=""
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Wno-unused-value $vf $sched -I include "$@" --cuda-device-only -S -o "$out" no-node-comparison_amd/csrc/$unit
