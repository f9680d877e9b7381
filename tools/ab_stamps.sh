#!/bin/bash
# Per-phase cycles of the config-2 solve (stamps build with sub-phases and the trial evaluation,
# libmpcx_sub2.so: tools/exp_build.sh) for the working tree and ab_base/, then the instruction-cost
# probe (tools/dpp_probe.hip, built beforehand).
set -o pipefail
mkdir -p gpurun_out/ab
for T in ab_base .; do
  n=$([ "$T" = . ] && echo new || echo base)
  MPCX_STAMPS_LIB=$PWD/$T/mpc-verde_amd/mpcx/libmpcx_sub2.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 200 \
    python3 tools/stamp_profile.py --steps 3 > gpurun_out/ab/stamps_$n.json 2> gpurun_out/ab/stamps_$n.err || exit 1
done
timeout -k 10 60 tools/dpp_probe > gpurun_out/dpp_probe.json || exit 1
cat gpurun_out/dpp_probe.json
