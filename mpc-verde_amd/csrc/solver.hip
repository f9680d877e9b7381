// solver.hip -- model dispatch of the fused solve (kernels.h, one translation unit per model:
// solve_<model>.hip) and the RK4+Jacobian sweep kernel over B x N unicycle intervals.
//
// Replaces, for B independent instances at once, the reference's
//   sol = solver(x0=w0, lbx, ubx, lbg, ubg, p)     Casadi/multiple_shooting_casadi.py:235-242
// (DESIGN.md §3), and the function + Jacobian evaluations IPOPT requests from CasADi (§4).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "solver.h"
#include "unicycle.h"

namespace mpcx {

// ------------------------------------------------------------------------------
// RK4 + Jacobian sweep over B x N unicycle intervals, tiled structure of arrays.
// One thread per instance walks its N intervals: X_{k+1} loaded for interval k stays in
// registers as interval k+1's X_k and x_ref is loaded once, so HBM sees exactly the
// compulsory bytes (reads (N+1)*3 + 2N + 3 doubles, writes 24N doubles per instance;
// DESIGN.md §4).  Layout: 64-instance tiles, tile index inside each stage (tix below), so
// every wave's loads/stores of one stage are contiguous 512-B rows of one block -- the
// store pattern HBM absorbs fastest on this part (tools/hbm_probe.hip).
// ------------------------------------------------------------------------------
constexpr int kRec = 24;  // fields of the per-stage sweep record
__device__ __forceinline__ size_t tix(int stage, int F, int i, long b, long T) {
  return (((size_t)stage * T + (b >> 6)) * F + i) * 64 + (b & 63);
}
// record index of field PAIR j (fields 2j, 2j+1) in units of 16 B: inside a tile's 12 KB
// block of one stage, lane b%64 owns 16 contiguous bytes of each 1 KB pair row
__device__ __forceinline__ size_t jpix(int stage, int j, long b, long T) {
  return (((size_t)stage * T + (b >> 6)) * (kRec / 2) + j) * 64 + (b & 63);
}

__global__ __launch_bounds__(256) void rk4_sens_kernel(int B, int N, StageParams sp, const double* __restrict__ X,
                                                       const double* __restrict__ U, const double* __restrict__ XR,
                                                       double* __restrict__ J) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long T = ((long)B + 63) / 64;
  v2d* __restrict__ J2 = reinterpret_cast<v2d*>(J);
  double x[3], xr[3];
  const double ur[2] = {0.0, 0.0};
  const double lz[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    x[i] = X[tix(0, 3, i, b, T)];
    xr[i] = XR[tix(0, 3, i, b, T)];
  }
  for (int k = 0; k < N; ++k) {
    double u[2], xn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) xn[i] = X[tix(k + 1, 3, i, b, T)];
#pragma unroll
    for (int i = 0; i < 2; ++i) u[i] = U[tix(k, 2, i, b, T)];
    double xf[3], q, A[9], Bm[6], g[5], H[15];
    uni_derivs<false>(sp, x, u, xr, ur, lz, 1.0, xf, q, A, Bm, g, H);
    // one 24-field record per stage: c(3) q(1) A(9) B(6) grad q(5), stored as 12 field
    // pairs of 16 B per lane (1 KB per wave-instruction, nontemporal) -- a wave's whole
    // output of a stage is one contiguous 12 KB block
    double r[kRec];
#pragma unroll
    for (int i = 0; i < 3; ++i) r[i] = xf[i] - xn[i];
    r[3] = q;
#pragma unroll
    for (int i = 0; i < 9; ++i) r[4 + i] = A[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) r[13 + i] = Bm[i];
#pragma unroll
    for (int i = 0; i < 5; ++i) r[19 + i] = g[i];
#pragma unroll
    for (int j = 0; j < kRec / 2; ++j) {
      const v2d v = {r[2 * j], r[2 * j + 1]};
      __builtin_nontemporal_store(v, &J2[jpix(k, j, b, T)]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = xn[i];
  }
}

hipError_t launch_rk4_sens(int B, int N, const StageParams& sp, const double* X, const double* U, const double* XR,
                           double* J, hipStream_t stream) {
  const long blocks = ((long)B + 255) / 256;
  hipLaunchKernelGGL(rk4_sens_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, B, N, sp, X, U, XR, J);
  return hipGetLastError();
}

// workspace per thread: restoration (kernels.h RestoWs) for the unicycle and the ODE models, plus
// the chain stash of the 6-state bicycle; none elsewhere
int resto_ws_slots(int model, int nx, int nu) {
  if (model != 1 && (model < 3 || model > 5)) return 0;  // the models with kResto: unicycle (1), ODE (3-5)
  return RestoWs::slots(nx, nu) + (model == 4 ? chain_ws_slots(nx, nu) : 0);  // model 4: OdeModel<DynBicycle>::kWsStash
}

// ---- model dispatch (the entry points live in solve_<model>.hip) -------------------
#define MPCX_DECLARE(tag)                                                                                       \
  hipError_t launch_solve_##tag(const SolveArgs&, hipStream_t);                                                 \
  hipError_t launch_resume_##tag(const SolveArgs&, hipStream_t);                                                \
  hipError_t solve_shape_##tag(const SolveArgs&, int*, int*, const char**);                                     \
  hipError_t launch_plant_##tag(const SolveArgs&, const double*, double*, double*, hipStream_t);                \
  hipError_t launch_constraints_##tag(const SolveArgs&, const double*, double*, hipStream_t);                    \
  hipError_t launch_shift_##tag(const SolveArgs&, double*, const double*, double*, const double*, double*,       \
                                const double*, double*, hipStream_t);                                           \
  int diag_set_stamps_##tag(void*);                                                                             \
  int diag_set_counters_##tag(void*);
MPCX_DECLARE(unicycle)
MPCX_DECLARE(unicycle_xfree)
MPCX_DECLARE(unicycle_scan)
MPCX_DECLARE(linear4)
MPCX_DECLARE(linear5)
MPCX_DECLARE(linear4x2)
MPCX_DECLARE(kin_bicycle)
MPCX_DECLARE(dyn_bicycle)
MPCX_DECLARE(cartpole)

// horizons from which the unicycle's Riccati recursion runs as a log-depth scan (models.h
// UnicycleScanModel): ceil(log2(N+1)) = 5 combine levels cost about as much as 25 chain steps
constexpr int kUnicycleScanMinN = 25;
// diagnostic knob: MPCX_UNICYCLE_SCAN_MIN_N overrides it (A/B of the two instantiations).  Only
// a whole number in [1, 256] is taken (256: the scan never runs); anything else keeps the default.
static int unicycle_scan_min_n() {
  static const int n = [] {
    const char* e = getenv("MPCX_UNICYCLE_SCAN_MIN_N");
    if (!e || !*e) return kUnicycleScanMinN;
    char* end = nullptr;
    const long v = strtol(e, &end, 10);
    return (*end == '\0' && v >= 1 && v <= 256) ? (int)v : kUnicycleScanMinN;
  }();
  return n;
}

// unicycle, the linear-model shapes the reference's QPs need (4x1 lateral / cart-pole, 5x1
// cart-pole with the previous input as a state; 4x2 for two-input models), and the BASELINE's nonlinear ODE variants
#define MPCX_DISPATCH(a, FN, ...)                                                 \
  do {                                                                            \
    if ((a).model == 1)                                                           \
      return (a).N >= unicycle_scan_min_n() ? FN##_unicycle_scan(__VA_ARGS__)                              \
             : (a).xbnd ? FN##_unicycle(__VA_ARGS__) : FN##_unicycle_xfree(__VA_ARGS__);                       \
    if ((a).model == 2 && (a).nx == 4 && (a).nu == 1) return FN##_linear4(__VA_ARGS__); \
    if ((a).model == 2 && (a).nx == 5 && (a).nu == 1) return FN##_linear5(__VA_ARGS__); \
    if ((a).model == 2 && (a).nx == 4 && (a).nu == 2) return FN##_linear4x2(__VA_ARGS__); \
    if ((a).model == 3) return FN##_kin_bicycle(__VA_ARGS__);                     \
    if ((a).model == 4) return FN##_dyn_bicycle(__VA_ARGS__);                     \
    if ((a).model == 5) return FN##_cartpole(__VA_ARGS__);                        \
    return hipErrorInvalidValue;                                                  \
  } while (0)

hipError_t launch_solve(const SolveArgs& a, hipStream_t stream) { MPCX_DISPATCH(a, launch_solve, a, stream); }
hipError_t launch_resume(const SolveArgs& a, hipStream_t stream) { MPCX_DISPATCH(a, launch_resume, a, stream); }
hipError_t solve_shape(const SolveArgs& a, int* G, int* R, const char** kname) {
  MPCX_DISPATCH(a, solve_shape, a, G, R, kname);
}
hipError_t launch_plant(const SolveArgs& a, const double* U, double* XF, double* QF, hipStream_t stream) {
  MPCX_DISPATCH(a, launch_plant, a, U, XF, QF, stream);
}
hipError_t launch_constraints(const SolveArgs& a, const double* W, double* Gout, hipStream_t stream) {
  MPCX_DISPATCH(a, launch_constraints, a, W, Gout, stream);
}
hipError_t launch_shift(const SolveArgs& a, double* P, const double* W, double* W0, const double* L, double* L0,
                        const double* LX, double* LX0, hipStream_t stream) {
  MPCX_DISPATCH(a, launch_shift, a, P, W, W0, L, L0, LX, LX0, stream);
}

}  // namespace mpcx

#ifdef MPCX_STAMPS
// diagnostic build: every model unit holds its own copy of the buffer pointers
extern "C" int mpcx_diag_set_stamp_buffer(void* d_buf) {
  using namespace mpcx;
  return diag_set_stamps_unicycle(d_buf) | diag_set_stamps_unicycle_xfree(d_buf) | diag_set_stamps_unicycle_scan(d_buf) | diag_set_stamps_linear4(d_buf) | diag_set_stamps_linear5(d_buf) | diag_set_stamps_linear4x2(d_buf) |
         diag_set_stamps_kin_bicycle(d_buf) | diag_set_stamps_dyn_bicycle(d_buf) | diag_set_stamps_cartpole(d_buf);
}
extern "C" int mpcx_diag_set_counter_buffer(void* d_buf) {
  using namespace mpcx;
  return diag_set_counters_unicycle(d_buf) | diag_set_counters_unicycle_xfree(d_buf) | diag_set_counters_unicycle_scan(d_buf) | diag_set_counters_linear4(d_buf) | diag_set_counters_linear5(d_buf) | diag_set_counters_linear4x2(d_buf) |
         diag_set_counters_kin_bicycle(d_buf) | diag_set_counters_dyn_bicycle(d_buf) | diag_set_counters_cartpole(d_buf);
}
#endif
