#!/bin/bash
# A/B: the replicated evaluation's cross-half sums by ds_bpermute (libmpcx_bp.so) against
# v_permlane32_swap (current); probe; config-2 parity tests on the experiment library
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx
timeout -k 10 120 ./tools/mfma_f64_probe > gpurun_out/r04_mfma_probe5.json 2> gpurun_out/r04_mfma_probe5.err || exit 1
grep per_double gpurun_out/r04_mfma_probe5.json
AB="--no-cpu --no-roofline --no-reference-warm-start"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04g_cur$i.json 2>gpurun_out/r04g_cur$i.err || exit 1
  MPCX_LIB=$L/libmpcx_bp.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04g_bp$i.json 2>gpurun_out/r04g_bp$i.err || exit 1
done
for f in gpurun_out/r04g_*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);s=d['solve_kernel'];print('$f',d['value'],d['lockstep']['value'],s['us_per_ipm_iteration'],s['timed_launch_ms'],s['timed_group_iterations'],d['failed_instances'])"; done
MPCX_LIB=$L/libmpcx_bp.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard.py -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04g_t.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/r04g_t.log
