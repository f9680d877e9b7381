#!/bin/bash
# GPU tests, then an A/B/n of library builds on the config-2 bench: tools/gpu_t_ab.sh LIB...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/abn.sh "--no-reference-warm-start" 2 "$@"
