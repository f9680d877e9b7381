#!/bin/bash
# Round evidence (run on the GPU box from the repo root), each GPU step under its own limit:
#   1. the -m gpu suite                          -> gpurun_out/gputest_all.log
#   2. PMC characterisation of the solve kernel -> gpurun_out/solve_pmc/summary.json (tools/solve_pmc.sh)
#   3. default bench line                        -> gpurun_out/bench_default.json
#   4. kernel-trace --stats of the bench command -> gpurun_out/prof_bench/
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
STEP=${1:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  (cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > "$OUT/gputest_all.log" 2>&1)
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  bash "$R/tools/solve_pmc.sh" > "$OUT/solve_pmc.log" 2>&1
  (cd "$R" && timeout -k 10 400 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err")
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o bench -- \
    python3 "$R/bench.py" --no-cpu > "$OUT/bench_prof.log" 2>&1
fi
