#!/bin/bash
# GPU tests, then an A/B/n of library builds on a bench configuration:
#   ABARGS="--config 5" tools/gpu_t_ab.sh LIB...      (NOTEST=1 skips the tests)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/t.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
bash tools/abn.sh "${ABARGS:-} --no-reference-warm-start" 2 "$@"
