#!/bin/bash
# A/B of the working tree against ab_base/ on one box (bench args $1, workload of tools/bits_compare.py $2):
# bit-for-bit comparison of the two libraries' results, then alternating bench runs (tools/ab_tree.sh).
set -e
mkdir -p gpurun_out/ab
MPCX_LIB=$PWD/ab_base/mpc-verde_amd/mpcx/libmpcx.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py "$2" gpurun_out/ab/base.npz
timeout -k 10 200 python3 tools/bits_compare.py "$2" gpurun_out/ab/new.npz
python3 tools/bits_compare.py --diff gpurun_out/ab/base.npz gpurun_out/ab/new.npz || echo BITS_DIFFER
bash tools/ab_tree.sh "$1" 3 ab_base .
