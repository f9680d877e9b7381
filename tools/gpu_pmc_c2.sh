#!/bin/bash
# PMC passes of the config-2 solve kernel only (quick check): gpurun_out/solve_pmc/c2/summary.json
cd "$GRAFT_REPO_ROOT"
SOLVE_PMC_OUT=$GRAFT_REPO_ROOT/gpurun_out/solve_pmc/c2 SOLVE_PMC_ARGS="--config 2 --no-reference-warm-start" bash tools/solve_pmc.sh > gpurun_out/pmc_c2.log 2>&1
rc=$?; tail -5 gpurun_out/pmc_c2.log; exit $rc
