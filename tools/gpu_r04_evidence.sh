#!/bin/bash
# round-4 evidence at the current sources: bench line (default command), kernel-trace stats of the
# same command, config-2 phase stamps (stamps + sub-phase + trial-evaluation build), every bench
# configuration (tools/bench_all.sh), then the -m gpu suite
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mpc-verde_amd/mpcx
timeout -k 10 400 python3 bench.py > gpurun_out/r04_bench_line.json 2> gpurun_out/r04_bench_line.err || exit 1
echo bench ok; tail -c 300 gpurun_out/r04_bench_line.json
(cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1) || exit 1
echo prof ok
MPCX_STAMPS_LIB=$L/libmpcx_ste.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 tools/stamp_profile.py --steps 3 > gpurun_out/r04_stamps_c2_eval.json 2> gpurun_out/r04_stamps_c2_eval.err || exit 1
echo stamps ok
bash tools/bench_all.sh || exit 1
echo bench_all ok
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04_tests.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/r04_tests.log
