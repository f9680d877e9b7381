#!/bin/bash
# Every bench configuration of DESIGN.md §6 on one GPU -> gpurun_out/bench_all/*.json
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/bench_all
mkdir -p "$O"
cd "$R"
run() { local name=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu --no-roofline "$@" > "$O/$name.log" 2>&1; grep '^{' "$O/$name.log" | tail -1 > "$O/$name.json"; }
run c2 --config 2
run c3 --config 3
run c4 --config 4
run c5 --config 5
run c3_kin --config 3 --model kin_bicycle --steps 10 --warmup 2
run c4_dyn --config 4 --model dyn_bicycle --steps 10 --warmup 2
run c5_cp --config 5 --model cartpole --steps 10 --warmup 2
