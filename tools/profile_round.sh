#!/bin/bash
# Profiling passes committed under profiles/ (run on the GPU box from the repo root):
#   1. FETCH_SIZE and WRITE_SIZE of the rk4_sens sweep in separate PMC passes (B = 2^19, N = 20),
#      summarised by tools/pmc_summary.py (gfx950 corrections) -> gpurun_out/rk4_sens_pmc.json
#   2. kernel-trace --stats of the default bench command -> gpurun_out/prof_bench/
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- python3 "$R/bench.py" --profile-sweep-only --roofline-reps 5 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- python3 "$R/bench.py" --profile-sweep-only --roofline-reps 5 > "$OUT/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT/pmc_fetch" "$OUT/pmc_write" 524288 20 "$OUT/rk4_sens_pmc.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o bench -- python3 "$R/bench.py" --no-cpu > "$OUT/bench_prof.log" 2>&1
