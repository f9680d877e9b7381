#!/bin/bash
# Repeated short bench lines of one configuration (no CPU baseline / sweep): tools/bench_quick.sh REPS bench-args...
set -uo pipefail
R=$1; shift
for i in $(seq 1 "$R"); do
  timeout -k 10 200 python3 bench.py "$@" --no-cpu --no-roofline 2>/dev/null > /tmp/bq.json || exit 1
  python3 -c "import json;d=json.loads([l for l in open('/tmp/bq.json') if l.startswith('{')][-1]);print(d['value'],d['lockstep']['value'],d['solve_kernel']['us_per_ipm_iteration'],d['iters_max'],d['failed_instances'])"
done
