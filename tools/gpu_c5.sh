#!/bin/bash
# config-5 characterisation: stamps of the diagnostic build, then the solve-kernel PMC passes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-r04}
timeout -k 10 300 python3 tools/stamp_profile.py --model pend --N 100 --batch 2048 --steps 3 > gpurun_out/${T}_stamps_c5.json 2> gpurun_out/${T}_stamps_c5.err || exit 1
SOLVE_PMC_OUT=$GRAFT_REPO_ROOT/gpurun_out/solve_pmc/c5 SOLVE_PMC_ARGS="--config 5 --no-reference-warm-start" bash tools/solve_pmc.sh > gpurun_out/pmc_c5.log 2>&1 || exit 1
cat gpurun_out/${T}_stamps_c5.json
