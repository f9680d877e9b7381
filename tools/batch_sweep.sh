#!/bin/bash
# Solves/s against the per-GPU batch (one MI355X): config 2 and config 5 bench lines at several B
# -> gpurun_out/batch_sweep/*.json (DESIGN.md §6 batch-size table)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/batch_sweep
mkdir -p "$O"
cd "$R"
for spec in "2 256" "2 512" "2 1024" "2 2048" "2 4096" "2 8192" "2 16384" "5 512" "5 1024" "5 2048" "5 4096" "5 8192"; do
  set -- $spec
  timeout -k 10 300 python3 bench.py --config "$1" --batch "$2" --no-cpu --no-roofline > "$O/c$1_b$2.log" 2>&1 || exit 1
  grep '^{' "$O/c$1_b$2.log" | tail -1 > "$O/c$1_b$2.json"
  python3 -c "import json;d=json.load(open('$O/c$1_b$2.json'));sk=d['solve_kernel'];print('config $1 B=$2', d['value'], d['lockstep']['value'], sk['us_per_ipm_iteration'], sk.get('group_size'), sk.get('replicas'))"
done
