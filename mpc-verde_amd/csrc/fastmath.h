// fastmath.h -- fp64 log and exp for the solve kernel's barrier and line-search terms (gfx950).
//
// The device library's log and exp are double-double evaluations of ~100 and ~60 FP64 VALU
// instructions.  The kernel's line search needs four of them per IPM iteration (the barrier
// log-sums of the current and trial points, the switching condition's theta^s_theta / (-gd)^s_phi),
// group-uniform or per lane, all on the issue-bound path.  These are the classic
// single-precision-free argument reductions with a minimax polynomial (Sun's fdlibm e_log.c /
// e_exp.c algorithms, restated; error below 1 ulp there), with the one division each takes
// formed by v_rcp_f64 and two Newton steps: ~30 and ~25 instructions, error <= 2 ulp (measured
// against the library on 10^6 arguments over the whole range, tests/test_gpu_stage.py).  Special
// arguments (0, inf, nan, under/overflow) are handled by selects and clamps, not by a fallback to
// the library routine.
//
// The C++ CPU restatement (test infrastructure) keeps std::log / std::pow: the kernel's barrier terms already
// differ from it at the ulp level (one log of a mantissa product per lane, kernels.h
// barrier_logsum), and the iteration counts are compared against it (tests/test_gpu_parity.py).
#pragma once
#include <hip/hip_runtime.h>

#include "collectives.h"

namespace mpcx {

constexpr double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10;

// log(x) for a finite x > 0 (subnormals included: frexp normalises them); no library fallback, so
// no second code path holds registers
__device__ __forceinline__ double log_fd_pos(double x) {
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int k = __builtin_amdgcn_frexp_exp(x);
  if (m < 0.70710678118654752440) {  // m in [sqrt(1/2), sqrt(2))
    m *= 2.0;
    k -= 1;
  }
  const double f = m - 1.0;  // exact (Sterbenz)
  const double s = f * rcp64(2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * fma(w, fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01), 3.999999999940941908e-01);
  const double t2 =
      z * fma(w, fma(w, fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01), 2.857142874366239149e-01),
              6.666666666666735130e-01);
  const double R = t2 + t1, hfsq = 0.5 * f * f, dk = (double)k;
  return dk * kLn2Hi - ((hfsq - fma(s, hfsq + R, dk * kLn2Lo)) - f);
}

// log(x) for any x with IEEE's special values by selects: log(0) = -inf, log(inf) = inf, log(x < 0)
// = log(nan) = nan -- no library fallback, whose second code path would hold registers where the
// kernel calls this (measured: a guarded version cost config 2 several per cent).  The special
// values matter: a line-search trial point whose slack rounds to exactly 0 (a bound of |b| = 200
// at mu = 1e-9) must get phi = +inf and be rejected, not a finite barrier term.
__device__ __forceinline__ double log_fd(double x) {
  const double r = log_fd_pos(x);
  return x > 0.0 ? (x == INFINITY ? INFINITY : r) : (x == 0.0 ? -INFINITY : NAN);
}

// exp(x), any x: the argument is clamped to [-1100, 1100] (exp underflows to 0 / overflows to inf
// there already; nan passes through), and ldexp rounds the subnormal range correctly
__device__ __forceinline__ double exp_fd(double x) {
  x = x < -1100.0 ? -1100.0 : (x > 1100.0 ? 1100.0 : x);
  const double kd = rint(x * 1.44269504088896338700);
  const double hi = fma(-kd, kLn2Hi, x), lo = kd * kLn2Lo;  // x - k ln2 (hi exact: |k| < 2^11)
  const double r = hi - lo, t = r * r;
  const double c =
      r - t * fma(t, fma(t, fma(t, fma(t, 4.13813679705723846039e-08, -1.65339022054652515390e-06),
                                  6.61375632143793436117e-05),
                          -2.77777777770155933842e-03),
                  1.66666666666666019037e-01);
  const double y = 1.0 - ((lo - (r * c) * rcp64(2.0 - c)) - hi);
  return __builtin_amdgcn_ldexp(y, (int)kd);
}

}  // namespace mpcx
