set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r05b/tests.log 2>&1 || { tail -60 gpurun_out/r05b/tests.log; exit 1; }
tail -8 gpurun_out/r05b/tests.log
tools/ab.sh mpc-verde_amd/mpcx/libmpcx.so mpc-verde_amd/mpcx/libmpcx_lds.so "--batch 2048" 2
tools/ab_tree.sh "" 2
