#!/bin/bash
# A/B of a run-time knob on one box, alternating runs of the same tree: tools/ab_env.sh "bench args" reps "VAR=value"
set -uo pipefail
ARGS=$1; R=${2:-2}; KNOB=$3
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for n in default knob; do
    if [ "$n" = knob ]; then E="env $KNOB"; else E=""; fi
    timeout -k 10 240 $E python3 bench.py $ARGS --no-cpu --no-roofline > gpurun_out/ab/env_${n}_$i.json 2> gpurun_out/ab/env_${n}_$i.err || exit 1
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab/env_${n}_$i.json') if l.startswith('{')][-1]);print('$n', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'], d['solve_kernel'].get('group_size'))"
  done
done
