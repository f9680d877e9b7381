set -o pipefail
mkdir -p gpurun_out/r05f
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_stage.py > gpurun_out/r05f/stage.log 2>&1; tail -2 gpurun_out/r05f/stage.log
tools/ab.sh mpc-verde_amd/mpcx/libmpcx.so mpc-verde_amd/mpcx/libmpcx_tay.so "" 2
tools/ab_tree.sh "" 2 ab_m2 . && mkdir -p gpurun_out/ab2 && cp gpurun_out/ab/*.json gpurun_out/ab2/ && tools/ab_tree.sh "--config 5" 2 ab_base0 ab_m2 .
