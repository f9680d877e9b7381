#!/bin/bash
# A/B of the working tree against ab_base/ (tools/base_build.sh) on one box, alternating runs:
#   tools/ab_tree.sh "bench args" reps
set -uo pipefail
ARGS=$1; R=${2:-2}
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for T in ab_base .; do
    n=$([ "$T" = . ] && echo new || echo base)
    timeout -k 10 240 python3 "$T/bench.py" $ARGS --no-cpu --no-roofline \
      > gpurun_out/ab/${n}_$i.json 2> gpurun_out/ab/${n}_$i.err || exit 1
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab/${n}_$i.json') if l.startswith('{')][-1]);print('$n', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'])"
  done
done
