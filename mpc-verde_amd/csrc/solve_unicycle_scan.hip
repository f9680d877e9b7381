// solve_unicycle_scan.hip -- UnicycleModel with the log-depth Riccati scan, launched for horizons N >= kUnicycleScanMinN (solver.hip).
#include "kernels.h"

MPCX_INSTANTIATE(UnicycleScanModel, unicycle_scan, "mpcx::UnicycleScanModel")
