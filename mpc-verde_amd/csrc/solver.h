// solver.h -- device-side launch interface shared by solver.hip and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "unicycle.h"

namespace mpcx {

struct SolveArgs {
  int B, N, max_iter, p_layout;
  int p_stride;
  double tol;
  StageParams sp;
  const double* P;      // B x p_stride (device)
  const double* w0;     // B x nw or null (cold start: X_k = x0, U = 0)
  const double* lam0;   // B x ng initial constraint multipliers or null
  const double* lamx0;  // B x nw initial bound multipliers (zU - zL) or null
  int warm;             // 1: IPOPT warm_start_init_point (multipliers given)
  double mu_init, bound_push, mult_push;
  const double* lbw;    // nw (device)
  const double* ubw;    // nw
  double* w_out;        // B x nw
  double* f_out;        // B or null
  double* lam_out;      // B x ng or null
  double* lamx_out;     // B x nw or null
  int32_t* status;      // B or null
  int32_t* iters;       // B or null
};

hipError_t launch_solve(const SolveArgs& a, hipStream_t stream);
hipError_t launch_rk4_sens(int B, int N, const StageParams& sp, const double* X, const double* U, const double* XR,
                           double* C, double* Q, double* A, double* Bm, double* G, hipStream_t stream);
hipError_t launch_plant(int B, int p_stride, int p_layout, const StageParams& sp, const double* P, const double* U,
                        double* XF, double* QF, hipStream_t stream);
hipError_t launch_shift(int B, int N, int p_stride, int p_layout, const StageParams& sp, double* P, const double* W,
                        double* W0, const double* L, double* L0, const double* LX, double* LX0, hipStream_t stream);

}  // namespace mpcx
