#!/bin/bash
# build an A/B variant of the library (same units and flags as build()): bash tools/build_ab.sh <name> -DFLAG=VAL ...
# (NONODE_SCHED="" builds nonode.hip with the default machine scheduler as well)
cd "$(dirname "$0")/.."
n=$1; shift
mkdir -p ab
python3 -c "import sys; import __graft_entry__ as g; g.compile_lib(sys.argv[1], defines=sys.argv[2:])" "ab/lib_$n.so" "$@"
