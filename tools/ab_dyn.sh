#!/bin/bash
# A/B of the 6-state bicycle against ab_base/: bit comparison of a cold batch + 3-step loop
# (tools/bits_compare.py dyn), then alternating config-4-dyn bench runs (tools/ab_tree.sh).
set -euo pipefail
mkdir -p gpurun_out/ab
MPCX_LIB=$PWD/ab_base/mpc-verde_amd/mpcx/libmpcx.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/bits_compare.py dyn gpurun_out/ab/dyn_base.npz
timeout -k 10 300 python3 tools/bits_compare.py dyn gpurun_out/ab/dyn_new.npz
python3 tools/bits_compare.py --diff gpurun_out/ab/dyn_base.npz gpurun_out/ab/dyn_new.npz || true
bash tools/ab_tree.sh "--config 4 --model dyn_bicycle --steps 10 --warmup 2" "${1:-2}" ab_base .
