#!/bin/bash
# round-4 first GPU pass: MFMA f64 probe, bench line, kernel-trace stats of the bench command,
# config-2 stamps (chain, and the scan instantiation at N = 20), then the -m gpu suite
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 120 ./tools/mfma_f64_probe > gpurun_out/r04_mfma_probe.json 2> gpurun_out/r04_mfma_probe.err || exit 1
echo probe ok
timeout -k 10 400 python3 bench.py > gpurun_out/r04_b1.json 2> gpurun_out/r04_b1.err || exit 1
tail -c 1500 gpurun_out/r04_b1.json
(cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1) || exit 1
echo prof ok
timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/r04_stamps_c2.json 2> gpurun_out/r04_stamps_c2.err || exit 1
MPCX_UNICYCLE_SCAN_MIN_N=20 timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/r04_stamps_c2_scan.json 2> gpurun_out/r04_stamps_c2_scan.err || exit 1
echo stamps ok
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04_t1.log 2>&1
echo "pytest rc=$?"
tail -5 gpurun_out/r04_t1.log
