#!/bin/bash
# round-4 MFMA-chain pass: probe, -m gpu suite on the new library, A/B bench against the HEAD build
# (libmpcx_head.so), then the default bench line
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mfma_f64_probe > gpurun_out/r04_mfma_probe2.json 2> gpurun_out/r04_mfma_probe2.err || exit 1
tail -2 gpurun_out/r04_mfma_probe2.json
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_stage.py -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04_stage.log 2>&1
rc=$?
echo "stage rc=$rc"; tail -25 gpurun_out/r04_stage.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread -x > gpurun_out/r04_t2.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/r04_t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AB="--no-cpu --no-roofline --no-reference-warm-start"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04_ab_new$i.json 2>gpurun_out/r04_ab_new$i.err || exit 1
  MPCX_LIB=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx/libmpcx_head.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 bench.py $AB > gpurun_out/r04_ab_head$i.json 2>gpurun_out/r04_ab_head$i.err || exit 1
done
for f in gpurun_out/r04_ab_*.json; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['lockstep']['value'],d['solve_kernel']['us_per_ipm_iteration'],d['solve_kernel']['timed_launch_ms'],d['solve_kernel']['timed_group_iterations'])"; done
timeout -k 10 400 python3 bench.py > gpurun_out/r04_b1.json 2> gpurun_out/r04_b1.err || exit 1
tail -c 600 gpurun_out/r04_b1.json
