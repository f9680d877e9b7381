#!/bin/bash
# PMC characterisation of the fused solve kernel (run on the GPU box from the repo root):
#   pass A: SQ wave-cycle breakdown (issuing / dependency-stalled / waiting) + instruction mix
#   pass B: FP64 VALU instruction counts + GRBM_GUI_ACTIVE
#   pass C: kernel-trace durations of the same command
# -> gpurun_out/solve_pmc/{a,b,trace}, summarised by tools/solve_pmc_summary.py
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${SOLVE_PMC_OUT:-$R/gpurun_out/solve_pmc}
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS=(--mode lockstep --steps 5 --warmup 2 --no-cpu --no-roofline ${SOLVE_PMC_ARGS:-})
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$OUT/a" -o pmc -- python3 "$R/bench.py" "${ARGS[@]}" \
  > "$OUT/a.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
  SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/b" -o pmc -- python3 "$R/bench.py" "${ARGS[@]}" \
  > "$OUT/b.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/trace.log" 2>&1
if [ -z "${SOLVE_PMC_NOSUMMARY:-}" ]; then
  python3 "$R/tools/solve_pmc_summary.py" "$OUT" > "$OUT/summary.json"
  cat "$OUT/summary.json"
fi
echo "solve_pmc: $OUT done"
