#!/bin/bash
# final round-4 check at HEAD: smoke, the -m gpu suite, the default bench line (with the round-4
# PMC record beside its roofline)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { tail -20 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04_tests_final.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r04_tests_final.log
timeout -k 10 400 python3 bench.py > gpurun_out/r04_bench_line_final.json 2> gpurun_out/r04_bench_line_final.err || exit 1
tail -c 400 gpurun_out/r04_bench_line_final.json
