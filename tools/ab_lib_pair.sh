set -o pipefail
mkdir -p gpurun_out/ab
L0=$PWD/mpc-verde_amd/mpcx/libmpcx.so; L1=$PWD/mpc-verde_amd/mpcx/libmpcx_nolicm.so
MPCX_LIB=$L0 MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py c2 gpurun_out/ab/base.npz || exit 1
MPCX_LIB=$L1 MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py c2 gpurun_out/ab/new.npz || exit 1
python3 tools/bits_compare.py --diff gpurun_out/ab/base.npz gpurun_out/ab/new.npz || echo BITS_DIFFER
bash tools/ab.sh $L0 $L1 "" 3
