#!/bin/bash
# A/B: config 2 with the Riccati chain (current library) against the log-depth scan in a
# state-bound-free, replicated instantiation (libmpcx_xs.so, MPCX_UNICYCLE_SCAN_MIN_N=20)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx
AB="--no-cpu --no-roofline --no-reference-warm-start"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04f_chain$i.json 2>gpurun_out/r04f_chain$i.err || exit 1
  MPCX_LIB=$L/libmpcx_xs.so MPCX_ALLOW_STALE_LIB=1 MPCX_UNICYCLE_SCAN_MIN_N=20 timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04f_scan$i.json 2>gpurun_out/r04f_scan$i.err || exit 1
done
# config 5 (cart-pole QP, N = 100, two-wave groups) at two waves per SIMD (amdgpu_waves_per_eu(2),
# libmpcx_w2.so) against one
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config 5 $AB > gpurun_out/r04f_c5one$i.json 2>gpurun_out/r04f_c5one$i.err || exit 1
  MPCX_LIB=$L/libmpcx_w2.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 bench.py --config 5 $AB > gpurun_out/r04f_c5two$i.json 2>gpurun_out/r04f_c5two$i.err || exit 1
done
for f in gpurun_out/r04f_*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);s=d['solve_kernel'];print('$f',d['value'],d['lockstep']['value'],s['us_per_ipm_iteration'],s['timed_launch_ms'],s['timed_group_iterations'],d['failed_instances'])"; done
