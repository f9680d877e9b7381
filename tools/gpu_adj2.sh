#!/bin/bash
# restoration/oracle-agreement tests after the 6-state derivative change, and the flop probe
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_resto.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/resto_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|differ from the C\+\+ oracle|Error|assert" gpurun_out/resto_tests.log | head -40
[ $rc -eq 0 ] || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -d gpurun_out/flops -o flops --output-format csv -- python3 tools/flop_probe.py > gpurun_out/flops.log 2>&1 || exit 1
python3 tools/flop_summary.py gpurun_out/flops > gpurun_out/r04_flop_probe.json && cat gpurun_out/r04_flop_probe.json
