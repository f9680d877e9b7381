#!/bin/bash
# sub-phase stamps of config 2: HEAD's VALU chain (libmpcx_sto.so) against the MFMA chain (libmpcx_stn.so)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in sto stn; do
    MPCX_STAMPS_LIB=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx/libmpcx_$v.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/r04_sub_${v}$i.json 2> gpurun_out/r04_sub_${v}$i.err || exit 1
  done
done
for f in gpurun_out/r04_sub_*.json; do echo $f; python3 -c "
import json;d=json.load(open('$f'));print({k:v for k,v in d.items() if k in ('cycles_per_iteration','share','iters')})"; done
