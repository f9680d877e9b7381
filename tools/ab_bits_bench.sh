#!/bin/bash
# A/B of the working tree against ab_base/ (tools/base_build.sh): the row-chain harness test, the
# bit-for-bit comparison of both libraries on a workload of tools/bits_compare.py ($1, default c2),
# then alternating bench runs (tools/ab_tree.sh, bench args $2).
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_rowchain.py > gpurun_out/rowchain_test.log 2>&1 || { tail -30 gpurun_out/rowchain_test.log; exit 1; }
tail -3 gpurun_out/rowchain_test.log
MPCX_LIB=$PWD/ab_base/mpc-verde_amd/mpcx/libmpcx.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py ${1:-c2} gpurun_out/ab/base.npz || exit 1
timeout -k 10 200 python3 tools/bits_compare.py ${1:-c2} gpurun_out/ab/new.npz || exit 1
python3 tools/bits_compare.py --diff gpurun_out/ab/base.npz gpurun_out/ab/new.npz || echo BITS_DIFFER
bash tools/ab_tree.sh "${2:-}" 3 ab_base .
