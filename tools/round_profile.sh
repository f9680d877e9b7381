#!/bin/bash
# Round evidence (run on the GPU box from the repo root), each GPU step under its own limit:
#   tests: the -m gpu suite                                   -> gpurun_out/gputest_all.log
#   pmc:   PMC characterisation of the solve kernel, config 2 and the config-5 swing-up
#          (tools/solve_pmc.sh)                               -> gpurun_out/solve_pmc{,_cp}/summary.json
#   bench: default bench line + kernel-trace --stats of the same command
#                                                             -> gpurun_out/bench_default.json, prof_bench/
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
for STEP in "$@"; do
  case "$STEP" in
    tests)
      (cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        > "$OUT/gputest_all.log" 2>&1) ;;
    pmc)
      bash "$R/tools/solve_pmc.sh" > "$OUT/solve_pmc.log" 2>&1
      SOLVE_PMC_OUT=$OUT/solve_pmc_cp SOLVE_PMC_ARGS="--config 5 --model cartpole" \
        bash "$R/tools/solve_pmc.sh" > "$OUT/solve_pmc_cp.log" 2>&1 ;;
    bench)
      (cd "$R" && timeout -k 10 400 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err")
      (cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof_bench" -o bench -- python3 "$R/bench.py" --no-cpu > "$OUT/bench_prof.log" 2>&1) ;;
  esac
done
