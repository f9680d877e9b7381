#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04_t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/r04_t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r04_b1.json 2> gpurun_out/r04_b1.err
echo "bench rc=$?"
tail -c 3000 gpurun_out/r04_b1.json
