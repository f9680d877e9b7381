#!/bin/bash
# The GPU steps that regenerate a round's evidence under profiles/ (run on the GPU box from the
# repo root: gpurun -- 'bash tools/round_profile.sh STEP...'), each under its own time limit; the
# script stops at the first step that fails.  Outputs go to gpurun_out/ (copy what is committed
# into profiles/rNN_*, see profiles/README.md):
#   smoke    __graft_entry__.smoke()                                -> gpurun_out/smoke.log
#   tests    the -m gpu suite                                       -> gpurun_out/gputest_all.log
#   bench    default bench line + kernel-trace --stats of the same command
#                                                                   -> gpurun_out/bench_default.json, prof_bench/
#   benchall every bench configuration (tools/bench_all.sh)        -> gpurun_out/bench_all/
#   pmc      PMC characterisation of every workload's solve kernel (tools/solve_pmc_all.sh)
#                                                                   -> gpurun_out/solve_pmc/summary.json
#   sweep    FETCH_SIZE / WRITE_SIZE passes of the rk4_sens sweep   -> gpurun_out/rk4_sens_pmc.json
#   stamps   per-phase cycles of the diagnostic builds (libmpcx_sub2.so: config 2 with sub-phases and
#            the trial evaluation; libmpcx_sub5.so: config 5 with sub-phases; build them with
#            `make -C mpc-verde_amd stamps` and tools/exp_build.sh, see tools/stamp_profile.py)
#                                                                   -> gpurun_out/stamps_c2_sub.json, stamps_c5_sub.json
#   traffic  FETCH_SIZE / WRITE_SIZE passes of the bench's timed solve launch -> gpurun_out/solve_traffic.json
#   flops    FP64 flops per unit of the building blocks (tools/flop_probe.py under --pmc)
#                                                                   -> gpurun_out/flop_probe.json
# A/B comparisons of source trees are tools/ab_tree.sh (trees from tools/base_build.sh).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
L=$R/mpc-verde_amd/mpcx
mkdir -p "$OUT"
for STEP in "$@"; do
  echo "== $STEP"
  case "$STEP" in
    smoke)
      (cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1)
      tail -1 "$OUT/smoke.log" ;;
    tests)
      (cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread > "$OUT/gputest_all.log" 2>&1) || { grep -E "FAILED|passed|failed" "$OUT/gputest_all.log" | tail; exit 1; }
      tail -1 "$OUT/gputest_all.log" ;;
    bench)
      (cd "$R" && timeout -k 10 400 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err")
      tail -c 400 "$OUT/bench_default.json"
      (cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof_bench" -o bench -- python3 "$R/bench.py" --no-cpu > "$OUT/bench_prof.log" 2>&1) ;;
    benchall)
      bash "$R/tools/bench_all.sh" ;;
    pmc)
      bash "$R/tools/solve_pmc_all.sh" > "$OUT/solve_pmc_all.log" 2>&1 ;;
    sweep)
      (cd /tmp && export TMPDIR=/tmp &&
        timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- \
          python3 "$R/bench.py" --profile-sweep-only --roofline-reps 5 > "$OUT/pmc_fetch.log" 2>&1 &&
        timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- \
          python3 "$R/bench.py" --profile-sweep-only --roofline-reps 5 > "$OUT/pmc_write.log" 2>&1)
      python3 "$R/tools/pmc_summary.py" "$OUT/pmc_fetch" "$OUT/pmc_write" 524288 20 "$OUT/rk4_sens_pmc.json" ;;
    stamps)
      (cd "$R" && MPCX_STAMPS_LIB=$L/libmpcx_sub2.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 \
        python3 tools/stamp_profile.py --steps 3 > "$OUT/stamps_c2_sub.json" 2> "$OUT/stamps_c2_sub.err")
      (cd "$R" && MPCX_STAMPS_LIB=$L/libmpcx_sub5.so MPCX_ALLOW_STALE_LIB=1 timeout -k 10 300 \
        python3 tools/stamp_profile.py --model pend --N 100 --batch 2048 --steps 3 > "$OUT/stamps_c5_sub.json" \
        2> "$OUT/stamps_c5_sub.err") ;;
    traffic)
      (cd /tmp && export TMPDIR=/tmp &&
        timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/solve_fetch" -o pmc -- \
          python3 "$R/bench.py" --profile-solve-only --no-cpu --no-roofline > "$OUT/solve_fetch.log" 2>&1 &&
        timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/solve_write" -o pmc -- \
          python3 "$R/bench.py" --profile-solve-only --no-cpu --no-roofline > "$OUT/solve_write.log" 2>&1)
      python3 "$R/tools/solve_traffic.py" "$OUT/solve_fetch" "$OUT/solve_write" "$OUT/solve_traffic.json" ;;
    flops)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
        SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/flops" -o flops -- \
        python3 "$R/tools/flop_probe.py" > "$OUT/flops.log" 2>&1)
      python3 "$R/tools/flop_summary.py" "$OUT/flops" > "$OUT/flop_probe.json" ;;
    *)
      echo "unknown step $STEP" >&2; exit 2 ;;
  esac
done
