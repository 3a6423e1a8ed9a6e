#!/bin/bash
# Diagnostic build with in-kernel s_memtime section stamps -> no-node-comparison_amd/libnonode_stamp.so
cd "$(dirname "$0")/.."
python3 -c "import __graft_entry__ as g; g.compile_lib('no-node-comparison_amd/libnonode_stamp.so', defines=['-DNONODE_STAMP=1'])"
