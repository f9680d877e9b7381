// flop_probe.hip -- per-unit FP64 work of the solve kernel's two per-node building blocks, for
// the algorithmic roofline (bench.py algorithmic_flops_per_group_iteration):
//   eval_probe    -- one stage evaluation Model::derivs (F, q, A, B, grad q and the Hessian of
//                    fs q + lam^T F) exactly as the solve kernel calls it (ODE models with their
//                    LDS value cache, as in the kernel);
//   riccati_probe -- one backward Riccati step riccati_step + riccati_gains with the model's
//                    structural masks and unit entries (riccati.h).
// One unit per thread, n a multiple of 64, so every lane of every wave holds a unit and the
// rocprofv3 FP64 instruction counts (tools/flop_probe.py) divide into flops per unit.
// Built into tests/hip/libflop_probe.so; not part of libmpcx.
#include "models.h"
#include "ode.h"
#include "riccati.h"

namespace mpcx {

// PASSES: the ODE models' hyper-dual pass derivatives (OdeModel::derivs_passes) instead of the
// path the kernel takes (tests/test_gpu_ode.py compares the 6-state bicycle's adjoint path to it)
template <class Model, bool PASSES = false>
__global__ void eval_probe_kernel(int n, ModelArgs ma, const double* Z, const double* L, const double* P, int pstride,
                                  double* out) {
  constexpr int NX = Model::NX, NU = Model::NU, NZ = NX + NU, NH = NZ * (NZ + 1) / 2;
  constexpr int NO = NX + 1 + NX * NX + NX * NU + NZ + NH;
  extern __shared__ double tcbuf[];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if constexpr (Model::kTrigSlots > 0) {
    ma.tc = tcbuf + threadIdx.x;
    ma.tc_stride = blockDim.x;
  }
  typename Model::Ctx c;
  Model::load_ctx(ma, i, P + (size_t)i * pstride, 0, true, c);
  double z[NZ], ln[NX];
  for (int j = 0; j < NZ; ++j) z[j] = Z[(size_t)i * NZ + j];
  for (int j = 0; j < NX; ++j) ln[j] = L[(size_t)i * NX + j];
  double xf[NX], q, A[NX * NX], Bm[NX * NU], g[NZ], H[NH];
  if constexpr (PASSES)
    Model::derivs_passes(ma, c, z, ln, 1.0, xf, q, A, Bm, g, H);
  else
    Model::derivs(ma, c, z, ln, 1.0, xf, q, A, Bm, g, H);
  double* o = out + (size_t)i * NO;
  int t = 0;
  for (int j = 0; j < NX; ++j) o[t++] = xf[j];
  o[t++] = q;
  for (int j = 0; j < NX * NX; ++j) o[t++] = A[j];
  for (int j = 0; j < NX * NU; ++j) o[t++] = Bm[j];
  for (int j = 0; j < NZ; ++j) o[t++] = g[j];
  for (int j = 0; j < NH; ++j) o[t++] = H[j];
}

// in per thread: Hd NH, gp NZ, A NX^2, B NX NU, c NX, P_{k+1} NP (packed), p_{k+1} NX
// out: P_k NP, p_k NX, K NU NX, k_f NU
template <class Model>
__global__ void riccati_probe_kernel(int n, const double* in, double* out) {
  constexpr int NX = Model::NX, NU = Model::NU, NZ = NX + NU, NH = NZ * (NZ + 1) / 2, NP = NX * (NX + 1) / 2;
  constexpr int NI = NH + NZ + NX * NX + NX * NU + NX + NP + NX, NO = NP + NX + NU * NX + NU;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* v = in + (size_t)i * NI;
  double Hd[NH], gp[NZ], A[NX * NX], Bm[NX * NU], c[NX], P[NP], p[NX];
  int t = 0;
  for (int j = 0; j < NH; ++j) Hd[j] = v[t++];
  for (int j = 0; j < NZ; ++j) gp[j] = v[t++];
  for (int j = 0; j < NX * NX; ++j) A[j] = v[t++];
  for (int j = 0; j < NX * NU; ++j) Bm[j] = v[t++];
  for (int j = 0; j < NX; ++j) c[j] = v[t++];
  for (int j = 0; j < NP; ++j) P[j] = v[t++];
  for (int j = 0; j < NX; ++j) p[j] = v[t++];
  // the structure the model's masks declare
  constexpr unsigned long long AONE = AOneOf<Model>::value;
  for (int j = 0; j < NX * NX; ++j) {
    if (!((Model::AMASK >> j) & 1ull)) A[j] = 0.0;
    if ((AONE >> j) & 1ull) A[j] = 1.0;
  }
  for (int j = 0; j < NX * NU; ++j)
    if (!((Model::BMASK >> j) & 1ull)) Bm[j] = 0.0;
  double Pn[NP], pn[NX], K[NU * NX], kf[NU];
  Fac<NX, NU> fac = {};
  (void)riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, false, AONE>(Hd, gp, A, Bm, c, P, p, Pn, pn, fac);
  riccati_gains<NX, NU>(fac, K, kf);
  double* o = out + (size_t)i * NO;
  t = 0;
  for (int j = 0; j < NP; ++j) o[t++] = Pn[j];
  for (int j = 0; j < NX; ++j) o[t++] = pn[j];
  for (int j = 0; j < NU * NX; ++j) o[t++] = K[j];
  for (int j = 0; j < NU; ++j) o[t++] = kf[j];
}

template <class Model, bool PASSES = false>
int launch_eval(int n, const ModelArgs& ma, const double* Z, const double* L, const double* P, int pstride, double* out) {
  const size_t lds = Model::kTrigSlots > 0 ? (size_t)Model::kTrigSlots * 64 * sizeof(double) : 0;
  hipLaunchKernelGGL((eval_probe_kernel<Model, PASSES>), dim3((n + 63) / 64), dim3(64), lds, 0, n, ma, Z, L, P, pstride,
                     out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return -1000 - (int)e;
  const hipError_t s = hipDeviceSynchronize();
  return s == hipSuccess ? 0 : -2000 - (int)s;
}
template <class Model>
int launch_riccati(int n, const double* in, double* out) {
  hipLaunchKernelGGL(riccati_probe_kernel<Model>, dim3((n + 63) / 64), dim3(64), 0, 0, n, in, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return -1000 - (int)e;
  const hipError_t s = hipDeviceSynchronize();
  return s == hipSuccess ? 0 : -2000 - (int)s;
}

}  // namespace mpcx

// model: 1 unicycle (cost 0 quadrature / 1 node), 3 kinematic bicycle, 4 dynamic bicycle,
// 5 cart-pole (include/mpcx.h model ids).  Z: n x NZ, L: n x NX, P: n x pstride (x0 then the
// reference), all device pointers; returns 0 on success.
static mpcx::ModelArgs probe_args(double T, int M, int cost, const double* Q, const double* R, const double* par) {
  using namespace mpcx;
  ModelArgs ma{};
  ma.p_layout = 0;
  ma.N = 1;
  ma.sp.T = T;
  ma.sp.M = M;
  ma.sp.h = T / M;
  ma.sp.cost = cost;
  for (int j = 0; j < 3; ++j) ma.sp.Q[j] = Q[j];
  for (int j = 0; j < 2; ++j) ma.sp.R[j] = R[j];
  ma.op.M = M;
  ma.op.h = T / M;
  for (int j = 0; j < 8; ++j) {
    ma.op.Q[j] = Q[j];
    ma.op.R[j] = R[j];
    ma.op.par[j] = par[j];
  }
  return ma;
}

extern "C" int eval_probe(int model, int n, double T, int M, int cost, const double* Q, const double* R,
                          const double* par, const double* Z, const double* L, const double* P, int pstride,
                          double* out) {
  using namespace mpcx;
  if (n <= 0 || n % 64 || M < 1) return -3;
  const ModelArgs ma = probe_args(T, M, cost, Q, R, par);
  switch (model) {
    case 1: return launch_eval<UnicycleModel>(n, ma, Z, L, P, pstride, out);
    case 3: return launch_eval<OdeModel<KinBicycle>>(n, ma, Z, L, P, pstride, out);
    case 4: return launch_eval<OdeModel<DynBicycle>>(n, ma, Z, L, P, pstride, out);
    case 5: return launch_eval<OdeModel<CartPole>>(n, ma, Z, L, P, pstride, out);
    default: return -4;
  }
}

// the ODE models through their hyper-dual passes (same arguments as eval_probe)
extern "C" int eval_probe_passes(int model, int n, double T, int M, int cost, const double* Q, const double* R,
                                 const double* par, const double* Z, const double* L, const double* P, int pstride,
                                 double* out) {
  using namespace mpcx;
  if (n <= 0 || n % 64 || M < 1) return -3;
  const ModelArgs ma = probe_args(T, M, cost, Q, R, par);
  switch (model) {
    case 3: return launch_eval<OdeModel<KinBicycle>, true>(n, ma, Z, L, P, pstride, out);
    case 4: return launch_eval<OdeModel<DynBicycle>, true>(n, ma, Z, L, P, pstride, out);
    case 5: return launch_eval<OdeModel<CartPole>, true>(n, ma, Z, L, P, pstride, out);
    default: return -4;
  }
}

extern "C" int riccati_probe(int model, int n, const double* in, double* out) {
  using namespace mpcx;
  if (n <= 0 || n % 64) return -3;
  switch (model) {
    case 1: return launch_riccati<UnicycleModel>(n, in, out);
    case 3: return launch_riccati<OdeModel<KinBicycle>>(n, in, out);
    case 4: return launch_riccati<OdeModel<DynBicycle>>(n, in, out);
    case 5: return launch_riccati<OdeModel<CartPole>>(n, in, out);
    case 41: return launch_riccati<LinearModel<4, 1>>(n, in, out);
    case 51: return launch_riccati<LinearModel<5, 1>>(n, in, out);
    default: return -4;
  }
}
