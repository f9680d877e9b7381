#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab.sh mpc-verde_amd/mpcx/libmpcx.so mpc-verde_amd/mpcx/libmpcx_r1.so "--no-reference-warm-start" 2 || exit 1
MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/r04_stamps_r2.json 2> gpurun_out/r04_stamps_r2.err || exit 1
tail -c 1500 gpurun_out/r04_stamps_r2.json
