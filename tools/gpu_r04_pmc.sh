#!/bin/bash
# round-4 PMC of every bench workload's solve kernel (tools/solve_pmc_all.sh) and the FP64 /
# cross-lane issue probe
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mfma_f64_probe > gpurun_out/r04_mfma_probe4.json 2> gpurun_out/r04_mfma_probe4.err || exit 1
tail -12 gpurun_out/r04_mfma_probe4.json
bash tools/solve_pmc_all.sh > gpurun_out/solve_pmc_all.log 2>&1 || { tail -20 gpurun_out/solve_pmc_all.log; exit 1; }
tail -3 gpurun_out/solve_pmc_all.log
