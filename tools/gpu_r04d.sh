#!/bin/bash
# MFMA chain (scaled) vs HEAD vs HEAD with one Newton step in the VALU chain: harness, A/B bench,
# sub-phase stamps, then the -m gpu suite
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_stage.py -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04d_stage.log 2>&1
rc=$?; echo "stage rc=$rc"; tail -3 gpurun_out/r04d_stage.log
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r04d_stage.log; exit $rc; fi
AB="--no-cpu --no-roofline --no-reference-warm-start"
for i in 1 2; do
  for v in head new nr1; do
    if [ $v = new ]; then E=""; else E="MPCX_LIB=$L/libmpcx_$v.so MPCX_ALLOW_STALE_LIB=1"; fi
    env $E timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04d_ab_$v$i.json 2>gpurun_out/r04d_ab_$v$i.err || exit 1
  done
done
for f in gpurun_out/r04d_ab_*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);s=d['solve_kernel'];print('$f',d['value'],d['lockstep']['value'],s['us_per_ipm_iteration'],s['timed_launch_ms'],s['timed_group_iterations'])"; done
for v in sto stn; do
  MPCX_STAMPS_LIB=$L/libmpcx_$v.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/r04d_sub_$v.json 2> gpurun_out/r04d_sub_$v.err || exit 1
done
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04d_t.log 2>&1
echo "pytest rc=$?"; tail -12 gpurun_out/r04d_t.log
