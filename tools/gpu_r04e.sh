#!/bin/bash
# A/B of the current library against the round-start build (libmpcx_head.so), probe, -m gpu suite
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx
T=${1:-e}
timeout -k 10 120 ./tools/mfma_f64_probe > gpurun_out/r04_mfma_probe3.json 2> gpurun_out/r04_mfma_probe3.err || exit 1
tail -9 gpurun_out/r04_mfma_probe3.json
AB="--no-cpu --no-roofline --no-reference-warm-start"
for i in 1 2 3; do
  for v in head new; do
    if [ $v = new ]; then E=""; else E="MPCX_LIB=$L/libmpcx_$v.so MPCX_ALLOW_STALE_LIB=1"; fi
    env $E timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04${T}_ab_$v$i.json 2>gpurun_out/r04${T}_ab_$v$i.err || exit 1
  done
done
for f in gpurun_out/r04${T}_ab_*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);s=d['solve_kernel'];print('$f',d['value'],d['lockstep']['value'],s['us_per_ipm_iteration'],s['timed_launch_ms'],s['timed_group_iterations'])"; done
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04${T}_t.log 2>&1
echo "pytest rc=$?"; tail -12 gpurun_out/r04${T}_t.log
