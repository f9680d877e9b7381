#!/bin/bash
# One A/B call of the working tree against ab_base/: row-chain harness, bit comparison (workload $1,
# default c2), per-phase stamps of both trees (libmpcx_sub2.so, if built), alternating bench runs
# (bench args $2).
set -o pipefail
mkdir -p gpurun_out/ab
bash tools/ab_bits_bench.sh "${1:-c2}" "${2:-}" || exit 1
for T in ab_base .; do
  n=$([ "$T" = . ] && echo new || echo base)
  [ -f $T/mpc-verde_amd/mpcx/libmpcx_sub2.so ] || continue
  MPCX_STAMPS_LIB=$PWD/$T/mpc-verde_amd/mpcx/libmpcx_sub2.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 \
    python3 tools/stamp_profile.py --steps 3 > gpurun_out/ab/stamps_$n.json 2> gpurun_out/ab/stamps_$n.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab/stamps_$n.json'));s=d['share'];c=d['cycles_per_iter'];print('$n', c, {k: round(v*c) for k,v in s.items() if v > 0.02})"
done
