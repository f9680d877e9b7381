#!/bin/bash
# Experiment build: recompile ONE model unit with extra flags and link it with the other units'
# current objects into mpc-verde_amd/mpcx/libmpcx_<tag>.so (load it with MPCX_LIB=... and
# MPCX_ALLOW_STALE_LIB=1).  A/B of compile-time switches without a full rebuild.
#   tools/exp_build.sh TAG UNIT [hipcc flags...]     e.g. tools/exp_build.sh ev unicycle_xfree -DMPCX_STAMP_EVAL
#   EXP_BASE=build/stamps tools/exp_build.sh st unicycle -DMPCX_STAMPS ...   (diagnostic-build variant)
set -euo pipefail
TAG=$1; UNIT=$2; shift 2
cd "$(dirname "$0")/../mpc-verde_amd"
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm -disable-machine-licm -mllvm -sink-insts-to-avoid-spills"  # as the Makefile (DEVFLAGS)
mkdir -p build/exp_$TAG
/opt/rocm/bin/hipcc $HIPFLAGS -I../include -Icsrc "$@" -c csrc/solve_$UNIT.hip -o build/exp_$TAG/solve_$UNIT.hip.o
BASE=${EXP_BASE:-build}  # build/stamps: link with the diagnostic build's objects
OBJS=""
for o in $BASE/*.o; do
  b=$(basename "$o")
  if [ "$b" = "solve_$UNIT.hip.o" ]; then OBJS="$OBJS build/exp_$TAG/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc $HIPFLAGS -shared $OBJS -o mpcx/libmpcx_$TAG.so
echo "mpc-verde_amd/mpcx/libmpcx_$TAG.so"
