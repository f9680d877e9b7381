#!/bin/bash
# 6-state bicycle adjoint derivatives: the ODE GPU tests, then A/B against the hyper-dual passes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ode.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/adj_tests.log 2>&1 || { tail -30 gpurun_out/adj_tests.log; exit 1; }
grep -E "PASS|FAIL|max relative" gpurun_out/adj_tests.log
bash tools/ab.sh mpc-verde_amd/mpcx/libmpcx.so mpc-verde_amd/mpcx/libmpcx_pas.so "--config 4 --model dyn_bicycle --steps 10 --warmup 2" 3
