#!/bin/bash
# A/B of libmpcx builds over the bench workloads on one box: bit comparison of configs 2, 5 and the
# 6-state bicycle against the first build (tools/bits_compare.py; the result files under /tmp:
# gpurun copies back at most 64 MiB), then alternating bench runs of each workload.
#   tools/ab_lib_all.sh "LIB_A LIB_B ..." [reps] [workloads: c2 c3 c4 c5 kin dyn cp]
set -o pipefail
LIBS=($1); R=${2:-2}; W=${3:-"c2 c3 c4 c5 kin dyn cp"}
name() { case "$1" in */mpc-verde_amd/mpcx/libmpcx.so) basename "$(dirname "$(dirname "$(dirname "$1")")")" ;; *) basename "$1" .so ;; esac; }
for w in c2 c5 dyn; do
  for L in "${LIBS[@]}"; do
    MPCX_LIB=$L MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 python3 tools/bits_compare.py $w /tmp/ab_bits_${w}_$(name $L).npz > /dev/null 2>&1 || exit 1
    [ "$L" = "${LIBS[0]}" ] && continue
    echo "bits $w $(name $L): $(python3 tools/bits_compare.py --diff /tmp/ab_bits_${w}_$(name ${LIBS[0]}).npz /tmp/ab_bits_${w}_$(name $L).npz | tr '\n' ' ' || echo DIFFER)"
  done
done
declare -A ARGS=([c2]="--config 2" [c3]="--config 3" [c4]="--config 4" [c5]="--config 5"
  [kin]="--config 3 --model kin_bicycle --steps 10 --warmup 2" [dyn]="--config 4 --model dyn_bicycle --steps 10 --warmup 2"
  [cp]="--config 5 --model cartpole --steps 10 --warmup 2")
for w in $W; do
  for i in $(seq 1 "$R"); do
    for L in "${LIBS[@]}"; do
      MPCX_LIB=$L MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 bench.py ${ARGS[$w]} --no-cpu --no-roofline > /tmp/ab_run.json 2> /tmp/ab_run.err || { tail /tmp/ab_run.err; exit 1; }
      python3 -c "import json;d=json.loads([l for l in open('/tmp/ab_run.json') if l.startswith('{')][-1]);print('$w', '$(name $L)', d['value'], d['lockstep']['value'], d['solve_kernel']['us_per_ipm_iteration'])"
    done
  done
done
