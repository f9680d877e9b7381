#!/bin/bash
# A/B of source trees on one box, alternating runs: tools/ab_tree.sh "bench args" reps TREE...
# (TREE = . for the working tree, or an ab_* directory made by tools/base_build.sh; default ab_base .)
set -uo pipefail
ARGS=$1; R=${2:-2}; shift 2 || true
TREES=("$@"); [ ${#TREES[@]} -eq 0 ] && TREES=(ab_base .)
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for T in "${TREES[@]}"; do
    n=$([ "$T" = . ] && echo new || echo "$T")
    timeout -k 10 240 python3 "$T/bench.py" $ARGS --no-cpu --no-roofline \
      > gpurun_out/ab/${n}_$i.json 2> gpurun_out/ab/${n}_$i.err || exit 1
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab/${n}_$i.json') if l.startswith('{')][-1]);print('$n', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'])"
  done
done
