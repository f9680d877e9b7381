#!/bin/bash
# PMC of the solve kernel for several libmpcx builds (one rocprofv3 --pmc pass each, lock-step
# bench run): tools/pmc_ab.sh "bench args" "COUNTERS" LIB...   -> gpurun_out/pmc_ab/<lib>/
set -uo pipefail
ARGS=$1; CNT=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename "$L" .so)
  O=$R/gpurun_out/pmc_ab/$n
  mkdir -p "$O"
  MPCX_LIB=$R/$L MPCX_ALLOW_STALE_LIB=1 timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$O" -o pmc -- \
    python3 "$R/bench.py" $ARGS --mode lockstep --no-cpu --no-roofline > "$O/run.log" 2>&1 || { echo "pmc failed for $n"; exit 1; }
  python3 "$R/tools/pmc_table.py" "$O" solve_kernel
done
