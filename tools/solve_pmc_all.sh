#!/bin/bash
# PMC characterisation of the solve kernel of every bench workload (configs 2-5 and the three
# nonlinear variants), one tools/solve_pmc.sh run per workload, merged into one JSON:
#   tools/solve_pmc_all.sh  ->  gpurun_out/solve_pmc/summary.json  (commit as profiles/r03_solve_kernel_pmc.json)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
B=$R/gpurun_out/solve_pmc
DIRS=()
run() {  # name, bench args
  SOLVE_PMC_OUT=$B/$1 SOLVE_PMC_ARGS="$2" SOLVE_PMC_NOSUMMARY=1 "$R/tools/solve_pmc.sh"
  DIRS+=("$B/$1")
}
run c2 "--config 2"
run c3 "--config 3"
run c4 "--config 4"
run c5 "--config 5"
run kin "--config 3 --model kin_bicycle"
run dyn "--config 4 --model dyn_bicycle"
run cartpole "--config 5 --model cartpole"
python3 "$R/tools/solve_pmc_summary.py" "${DIRS[@]}" > "$B/summary.json"
echo "wrote $B/summary.json"
