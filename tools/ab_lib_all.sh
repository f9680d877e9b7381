#!/bin/bash
# A/B of two libmpcx builds over the bench workloads on one box: bit comparison of configs 2, 5 and
# the 6-state bicycle (tools/bits_compare.py; the result files under /tmp: gpurun copies back at most 64 MiB), then alternating bench runs of each workload.
#   tools/ab_lib_all.sh LIB_A LIB_B [reps]
set -o pipefail
A=$1; B=$2; R=${3:-2}
mkdir -p gpurun_out/ab
for w in c2 c5 dyn; do
  for L in "$A" "$B"; do
    n=$(basename "$(dirname "$(dirname "$(dirname "$L")")")")_$(basename "$L" .so)
    MPCX_LIB=$L MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py $w /tmp/ab_bits_${w}_$n.npz > /dev/null 2>&1 || exit 1
  done
  echo "bits $w: $(python3 tools/bits_compare.py --diff /tmp/ab_bits_${w}_*.npz | tr '\n' ' ' || echo DIFFER)"
done
for args in "--config 2" "--config 3" "--config 4" "--config 5" "--config 3 --model kin_bicycle --steps 10 --warmup 2" "--config 4 --model dyn_bicycle --steps 10 --warmup 2" "--config 5 --model cartpole --steps 10 --warmup 2"; do
  for i in $(seq 1 "$R"); do
    for L in "$A" "$B"; do
      MPCX_LIB=$L MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 bench.py $args --no-cpu --no-roofline > gpurun_out/ab/run.json 2> gpurun_out/ab/run.err || exit 1
      python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab/run.json') if l.startswith('{')][-1]);print('$args'.replace('--',''), '$L'.split('/')[-4], d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'])"
    done
  done
done
