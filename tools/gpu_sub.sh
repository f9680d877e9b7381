#!/bin/bash
# sub-phase stamps (errors and Riccati split, -DMPCX_STAMP_SUB) of one model unit's experiment
# build: tools/gpu_sub.sh TAG LIB [stamp_profile args...]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=$1; LIB=$2; shift 2
MPCX_STAMPS_LIB=$LIB MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py "$@" > gpurun_out/${T}_sub.json 2> gpurun_out/${T}_sub.err || exit 1
cat gpurun_out/${T}_sub.json
