#!/bin/bash
# config-5 phase stamps at the round-4 sources: phases (stamps build) and sub-phases (-DMPCX_STAMP_SUB)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/stamp_profile.py --model pend --N 100 --batch 2048 --steps 3 > gpurun_out/r04h_stamps_c5.json 2> gpurun_out/r04h_stamps_c5.err || exit 1
MPCX_STAMPS_LIB=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx/libmpcx_c5sub.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py --model pend --N 100 --batch 2048 --steps 3 > gpurun_out/r04h_sub_c5.json 2> gpurun_out/r04h_sub_c5.err || exit 1
cat gpurun_out/r04h_stamps_c5.json gpurun_out/r04h_sub_c5.json
