#!/bin/bash
# A/B/n of libmpcx builds on one box (alternating runs): tools/abn.sh "bench args" reps LIB...
set -uo pipefail
ARGS=$1; R=$2; shift 2
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for L in "$@"; do
    n=$(basename "$L" .so)
    MPCX_LIB=$L MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 bench.py $ARGS --no-cpu --no-roofline \
      > gpurun_out/ab/${n}_$i.json 2> gpurun_out/ab/${n}_$i.err || exit 1
    python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/ab/${n}_$i.json') if l.startswith('{')][-1]);print('$n', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'], d['iters_mean'], d['solve_kernel']['timed_launch_ms'], d['solve_kernel']['timed_group_iterations'])"
  done
done
