set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullbatch.py tests/test_gpu_linear.py > gpurun_out/r05b/tests.log 2>&1 || { tail -60 gpurun_out/r05b/tests.log; exit 1; }
tail -30 gpurun_out/r05b/tests.log
tools/ab.sh mpc-verde_amd/mpcx/libmpcx.so mpc-verde_amd/mpcx/libmpcx_lds.so "--batch 2048" 2
