// kernels.h -- fused batched interior-point solve of multiple-shooting MPC NLPs on gfx950
// (MI355X), and the per-model plant / shift / constraint kernels.  Included by one
// translation unit per stage model (solve_<model>.hip, MPCX_INSTANTIATE), so the models
// compile in parallel; solver.hip holds the dispatch and the RK4+Jacobian sweep.
//
// Replaces, for B independent instances at once, the reference's
//   sol = solver(x0=w0, lbx, ubx, lbg, ubg, p)     Casadi/multiple_shooting_casadi.py:235-242
// where solver = ca.nlpsol('solver', 'ipopt', prob, opts) (:181-197) -- IPOPT's primal-dual
// barrier method (Waechter & Biegler 2006) on the NLP of :116-178 -- and the mpctools
// nmpc/QP solves of Trajectory_tracking.py:72,107 and inverted_pendulum_...py:64,74.
//
// Execution model: one *lane group* of G = 16/32/64 lanes per instance;
// lane k owns shooting node k: X_k, U_k, the defect of interval k, its multipliers, bound
// duals, the stage derivative blocks (A_k, B_k, g_k, H_k, all in VGPRs) and its Riccati
// data.  The whole solve -- evaluation sweep, KKT Riccati factor/solve, fraction-to-
// boundary, filter line search, barrier update -- runs inside ONE launch; nothing but the
// inputs and the solution touch HBM.  Node-parallel work runs on all lanes; the Riccati
// recursion and the forward roll-out are the sequential critical path and carry only
// what the next node needs (value function, state step) lane to lane by DPP.  Per-
// instance scalars are symmetric group reductions (bit-identical on every lane).  Every
// loop is wave-uniform; lanes of finished instances are predicated.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "collectives.h"
#include "fastmath.h"
#include "models.h"
#include "ode.h"
#include "pscan.h"
#include "riccati.h"
#include "rowchain.h"
#include "rowchain6.h"
#include "solver.h"

// Diagnostic build only (-DMPCX_STAMPS, `make stamps`): per-phase s_memtime cycle
// accounting of the solve loop (cdna_hip_programming.md §7 "In-kernel stamps").
#ifdef MPCX_STAMPS
static __device__ unsigned long long* g_mpcx_stamps = nullptr;
constexpr int kStampSlots = 16;  // per wave: phases 0-9, sub-phases 10-15 (-DMPCX_STAMP_SUB)
// per-instance event counters (diagnostic build; indices at the kernel's `diag` array)
static __device__ int* g_mpcx_diag = nullptr;
constexpr int kDiag = 15;  // counters per instance
#define DIAG(i) (++diag[(i)])
#define DIAG_IF(c, i) \
  do {                \
    if (c) ++diag[(i)]; \
  } while (0)
#define STAMP(p)                                                                \
  do {                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                          \
    unsigned long long t_;                                                      \
    asm volatile("s_memtime %0 ; stamp " #p "\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                          \
    st_acc[st_ph] += t_ - st_last;                                              \
    st_last = t_;                                                               \
    st_ph = (p);                                                                \
  } while (0)
#else
#define STAMP(p) \
  do {           \
  } while (0)
#endif
// finer split of the errors and Riccati phases (diagnostic build with -DMPCX_STAMP_SUB)
#if defined(MPCX_STAMPS) && defined(MPCX_STAMP_SUB)
#define STAMP_SUB(p) STAMP(p)
#else
#define STAMP_SUB(p) \
  do {               \
  } while (0)
#endif
#ifndef MPCX_STAMPS
#define DIAG(i) \
  do {          \
  } while (0)
#define DIAG_IF(c, i) \
  do {                \
  } while (0)
#endif

namespace mpcx {

// Model::kDecSuffix if the model declares it (linear models), false otherwise
template <class M, class = void>
struct DecSuffixOf {
  static constexpr bool value = false;
};
template <class M>
struct DecSuffixOf<M, std::void_t<decltype(M::kDecSuffix)>> {
  static constexpr bool value = M::kDecSuffix;
};

// IPOPT constants (Waechter & Biegler 2006 Table 1; IPOPT defaults)
constexpr double kEps = 2.220446049250313e-16;
constexpr double kKappaEps = 10.0, kKappaMu = 0.2, kThetaMu = 1.5, kTauMin = 0.99;
constexpr double kKappaSigma = 1e10, kSmax = 100.0;
constexpr double kGammaTheta = 1e-5, kGammaPhi = 1e-8, kDeltaSw = 1.0, kSTheta = 1.1, kSPhi = 2.3;
constexpr double kEtaPhi = 1e-8, kGammaAlpha = 0.05;
constexpr double kDw0 = 1e-4, kDwMin = 1e-20, kDwMax = 1e40, kKwMinus = 1.0 / 3, kKwPlus = 8, kKwPlusBar = 100;
constexpr double kBoundPush = 1e-2, kBoundFrac = 1e-2, kInfBound = 1e19;
constexpr int kFilterResetTrigger = 5, kMaxFilterResets = 5;  // IPOPT filter_reset_trigger, max_filter_resets

// interleaved reference layout w = [X_0 | U_0 X_1 | ... | U_{N-1} X_N]
template <int NX, int NU>
__device__ __forceinline__ int ixw(int k, int i) {
  return k == 0 ? i : NX + (NX + NU) * (k - 1) + NU + i;
}
template <int NX, int NU>
__device__ __forceinline__ int iuw(int k, int i) {
  return NX + (NX + NU) * k + i;
}

// workspace load through the global address space (a global_load, not a flat load that might
// alias the stack)
__device__ __forceinline__ double wsload(const double* base, long i) {
  return ((const __attribute__((address_space(1))) double*)base)[i];
}

// sum of log(slack) over the bounded components of a lane's variables as ONE log: the
// product of the slacks' frexp mantissas (each in [0.5, 1), at most 2 NZ factors, so no
// under/overflow) plus the exponents times ln 2.  One log instead of one per bound.
template <int NZ, class BL = const double*, class BU = const double*>
__device__ __forceinline__ double barrier_logsum(const double* z, const BL& lb, const BU& ub, const bool* hL,
                                                 const bool* hU) {
  double m = 1.0;
  int e = 0;
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    int el, eu;
    const double ml = frexp(z[i] - lb[i], &el), mu = frexp(ub[i] - z[i], &eu);
    m *= hL[i] ? ml : 1.0;
    e += hL[i] ? el : 0;
    m *= hU[i] ? mu : 1.0;
    e += hU[i] ? eu : 0;
  }
  return log_fd(m) + (double)e * 0.69314718055994530942;  // m = 0 (a slack at its bound): -inf
}

// IPOPT's filter (W&B 2006 §2.4, Filter::AddEntry) held in LDS by the lanes of a group: lane k
// owns entry slots k + G j, j < S = FilterLds<G>::S (S G >= 256 entries per instance); a free
// slot holds (+inf, +inf), so the membership test is plain `th >= th_j && ph >= ph_j`.  Entries
// are appended (slot n, no group collective) until all S G slots have been used; from then on an
// addition first drops the entries the new one dominates (as IPOPT's AddEntry does; a dominated
// entry never decides a test, so dropping it earlier would change nothing) and takes the lowest
// free slot, so the slots bound the filter only when more than S G entries are mutually
// non-dominated: then slot `next` (rotating) is overwritten and add() returns true (counted by
// the diagnostic build: DIAG 14).  Tests and updates touch the used rows only (one row while the
// filter holds at most G entries).  LDS rather than registers: the filter is read once per
// line-search trial and written once per iteration, and registers are the kernel's bottleneck.
template <int G>
struct FilterLds {
  static constexpr int kB = G > 64 ? G : 64;           // threads per block = column stride
  static constexpr int S = 256 / G > 2 ? 256 / G : 2;  // slot rows
  static constexpr int kCap = S * G;
  static constexpr int kDoubles = 2 * S * kB;          // LDS per block
  double* p;  // this thread's column of the block's buffer: th_j = p[2 j kB], ph_j = p[(2 j + 1) kB]
  int n;      // slots used (group-uniform); kCap once the filter has filled up
  int next;   // overflow slot (rotating)
  __device__ __forceinline__ double& th(int j) const { return p[(2 * j) * kB]; }
  __device__ __forceinline__ double& ph(int j) const { return p[(2 * j + 1) * kB]; }
  __device__ __forceinline__ int rows() const { return (n + G - 1) / G; }
  __device__ __forceinline__ void clear() {
    for (int j = 0; j < rows(); ++j) th(j) = ph(j) = INFINITY;
    n = next = 0;
  }
  __device__ __forceinline__ void init(double* col) {  // every slot (kernel start)
    p = col;
    n = kCap;
    clear();
  }
  // (t, q) lies in the region of one of this lane's entries
  __device__ __forceinline__ bool covers(double t, double q) const {
    bool r = false;
    for (int j = 0; j < rows(); ++j) r |= t >= th(j) && q >= ph(j);
    return r;
  }
  __device__ __forceinline__ bool contains(double t, double q, XWave<G>& xw) const {
    return n > 0 && gany<G>(covers(t, q), xw);
  }
  __device__ __forceinline__ bool add(double nth, double nph, int k, XWave<G>& xw) {
    if (n < kCap) {  // append
      if (n % G == k) {
        th(n / G) = nth;
        ph(n / G) = nph;
      }
      ++n;
      return false;
    }
    // full: drop what the new entry dominates, take the lowest free slot
    double low = (double)kCap;
    for (int j = 0; j < S; ++j)
      if (th(j) >= nth && ph(j) >= nph) {
        th(j) = ph(j) = INFINITY;
        low = fmin(low, (double)(k + G * j));
      }
    const int slot = (int)gmin<G>(low, xw);
    const bool ovf = slot >= kCap;
    const int put = ovf ? next : slot;
    if (put % G == k) {
      th(put / G) = nth;
      ph(put / G) = nph;
    }
    if (ovf) next = next + 1 == kCap ? 0 : next + 1;
    return ovf;
  }
};
static_assert(FilterLds<16>::S <= RestoWs::kFilterMax, "workspace slots of the filter");


}  // namespace mpcx
#include "resto.h"  // IPOPT's soft restoration and restoration phase (cold, out of line)
namespace mpcx {

// rarely taken branches: laid out away from the hot loop
#define MPCX_COLD(c) __builtin_expect(!!(c), 0)

// Model::kBoundsLds if the model declares it: the variable bounds of a lane live in LDS (its
// column of a per-block buffer) instead of 2 NZ doubles of registers held through every phase
template <class M, class = void>
struct BoundsLdsOf {
  static constexpr bool value = false;
};
template <class M>
struct BoundsLdsOf<M, std::void_t<decltype(M::kBoundsLds)>> {
  static constexpr bool value = M::kBoundsLds;
};

// read view of n doubles of a lane's LDS column (element i at p[i * S + off]).  relaunder()
// makes the offset opaque to the compiler at a phase boundary, so loads of one phase are never
// merged with (or hoisted into registers for) another phase: the values are re-read where used.
template <int S>
struct LdsCol {
  const double* p;
  int off;
  __device__ __forceinline__ double operator[](int i) const { return p[i * S + off]; }
  __device__ __forceinline__ void relaunder() { asm volatile("" : "+v"(off)); }
};

// Model::kRowChain if the model declares it: its sequential Riccati recursion runs as the row chain
// (rowchain.h) in the single-wave groups of 32 and 64 lanes
template <class M, class = void>
struct RowChainOf {
  static constexpr bool value = false;
};
template <class M>
struct RowChainOf<M, std::void_t<decltype(M::kRowChain)>> {
  static constexpr bool value = M::kRowChain;
};

// R = 2 (replicated groups, G = 32): a batch too small to give every SIMD a wave runs one
// instance per wave with its lane group held TWICE, in the wave's two 32-lane halves (replica rho
// = lane / 32).  Both replicas compute the same bits (every collective is a 32-lane group
// collective, as for two instances per wave); only replica 0 writes results.  The sequential
// phases split their work between the replicas.
template <class Model, int G, bool RESUME = false, int R = 1>
__global__ __launch_bounds__(G * R > 64 ? G * R : 64) void solve_kernel(SolveArgs a) {
  static_assert(R == 1 || (R == 2 && G == 32), "replicated groups: two 32-lane replicas per wave");
  constexpr int NX = Model::NX, NU = Model::NU, NZ = NX + NU, NH = NZ * (NZ + 1) / 2, NP = NX * (NX + 1) / 2;
  // resume launch: nothing parked by this step's solve launch -> return before any setup
  if constexpr (RESUME)
    if (*a.park_flag != a.park_epoch) return;
  static_assert(NP + NX <= kXchStride && 2 * NZ + NX <= kXchStride && NX * NX + NX <= kXchStride,
                "LDS exchange slot too small");
  const int lane = threadIdx.x & 63;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = (int)(gid & (G - 1));  // node of this lane
  // multi-wave groups (G > 64, one workgroup per instance) exchange through LDS
  __shared__ double xch[2 * XWave<G>::W * kXchStride];
  // LDS buffer of the Riccati scan (pscan.h): one element per thread, structure of arrays
  constexpr int kSBS = G > 64 ? G : 64;  // threads per block = field stride
  __shared__ double sbuf[Model::kParallelRiccati ? RElem<NX>::NE * kSBS : 1];
  // the 6-state row chain (rowchain6.h): one instance per wave, its node records in an LDS ring
  // that aliases the transcendental cache (idle during the Riccati phase)
  constexpr bool kRow6 = RowChainOf<Model>::value && rowchain6::fits<Model>() && G == 64 && R == 1;
  // LDS cache of the ODE models' transcendental values across their derivative passes (ode.h)
  constexpr int kTcache = Model::kTrigSlots > 0 ? Model::kTrigSlots * kSBS : 1;
  __shared__ double tcache[kRow6 && rowchain6::kRing > kTcache ? rowchain6::kRing : kTcache];
  // the decoupled suffix's vector scan (multi-wave groups): two NX-double buffers per thread, then
  // the matrix powers (A^T)^(j 4^l), j = 1..3, l < 5, kept for the launch (table index pow_tab)
  __shared__ double dscan[DecSuffixOf<Model>::value && G > 64 ? 2 * NX * kSBS + 15 * NX * NX : 1];
  double pow_tab = -1.0;  // table whose powers dscan holds (block-uniform)
  // the row chain's node records (rowchain.h): G records per instance of the wave
  constexpr bool kRow = RowChainOf<Model>::value && rowchain::fits<Model>() && G >= 32 && G * R <= 64;
  __shared__ double rcbuf[kRow ? (64 / (G * R)) * G * rowchain::kRec : 1];
  // workspace chain stash (solver.h chain_ws_slots): slots after the restoration workspace's
  constexpr bool kWsStash = WsStashOf<Model>::value;
  // The stash is one contiguous record per thread (array of structures, after the restoration
  // workspace's slot-major part): the chain's single active lane then reads its operands from
  // a few cache lines in 16-byte loads instead of one line per value.
  constexpr int kWsH = RestoWs::slots(NX, NU);  // slot-major slots before the records
  constexpr int kCS = chain_ws_slots(NX, NU);   // record: stage Hessian (NH), Sigma (NZ), A (NX^2), B (NX NU)
  constexpr int kRH = 0, kRS = NH, kRA = NH + NZ, kRB = NH + NZ + NX * NX, kRP = kRB + NX * NU;
  constexpr int kRZ = kRP + (NX + 1) * NX;  // the iterate across the row chain (stash below)
  static_assert(!kWsStash || (kRZ + 5 * NZ + NX == kCS && kCS % 2 == 0), "chain stash record");
  // this thread's record (16-byte aligned: hipMalloc base, 64-thread-multiple stride, even kCS);
  // opaque, so no address is hoisted out of the solve loop
  auto wsrec = [&]() __attribute__((always_inline)) -> const double* {
    double* r = a.ws + (long)kWsH * a.ws_stride + gid * kCS;
    asm volatile("" : "+v"(r));
    return (const double*)__builtin_assume_aligned(r, 16);
  };
  XWave<G> xw{xch, 0};
  const int inst = (int)(gid / (G * R));
  const int rho = R > 1 ? (int)((threadIdx.x / G) % R) : 0;  // replica of this lane (0: the writer)
  const bool valid = inst < a.B;
  const int N = a.N;
  const int nw = NX + NZ * N, ng = NX * (N + 1);
  const bool hasX = valid && k <= N;
  const bool hasU = valid && k < N;

  // ---- per-instance parameters and per-node model context
  double x0[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) x0[i] = 0.0;
  const double* Pin = a.P + (size_t)(valid ? inst : 0) * a.p_stride;
  if (valid)
#pragma unroll
    for (int i = 0; i < NX; ++i) x0[i] = Pin[i];
  const ModelArgs ma = [&] {
    ModelArgs m = model_args(a);
    if (Model::kTrigSlots > 0) {
      m.tc = tcache + threadIdx.x;
      m.tc_stride = kSBS;
    }
    return m;
  }();
  typename Model::Ctx ctx;
  Model::load_ctx(ma, valid ? inst : 0, Pin, k, hasU, ctx);

  // ---- bounds of my variables z = (x_k, u_k); x_0 is free (pinned by g_0)
  constexpr bool kBndLds = BoundsLdsOf<Model>::value;
  __shared__ double bndbuf[kBndLds ? 2 * NZ * kSBS : 1];
  double lb0[NZ], ub0[NZ];
  bool hL[NZ], hU[NZ];
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    lb0[i] = -1e20;
    ub0[i] = 1e20;
  }
  if (XBoundsOf<Model>::value && hasX && k > 0)
    for (int i = 0; i < NX; ++i) {
      lb0[i] = a.lbw[ixw<NX, NU>(k, i)];
      ub0[i] = a.ubw[ixw<NX, NU>(k, i)];
    }
  if (hasU)
    for (int i = 0; i < NU; ++i) {
      lb0[NX + i] = a.lbw[iuw<NX, NU>(k, i)];
      ub0[NX + i] = a.ubw[iuw<NX, NU>(k, i)];
    }
  int nbnd_l = 0;
  constexpr bool kXB = XBoundsOf<Model>::value;  // false: no state is bounded (compile-time)
#pragma unroll
  for (int i = 0; i < NZ; ++i) {
    const bool own = (i < NX) ? hasX : hasU;
    hL[i] = (kXB || i >= NX) && own && lb0[i] > -kInfBound;
    hU[i] = (kXB || i >= NX) && own && ub0[i] < kInfBound;
    nbnd_l += (int)hL[i] + (int)hU[i];
  }
  // lb / ub: registers, or (kBndLds) views of this lane's LDS column re-read in every phase
  using BndT = std::conditional_t<kBndLds, LdsCol<kSBS>, const double*>;
  BndT lb{}, ub{};
  if constexpr (kBndLds) {
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      bndbuf[i * kSBS + threadIdx.x] = lb0[i];
      bndbuf[(NZ + i) * kSBS + threadIdx.x] = ub0[i];
    }
    lb = LdsCol<kSBS>{bndbuf, (int)threadIdx.x};
    ub = LdsCol<kSBS>{bndbuf + NZ * kSBS, (int)threadIdx.x};
  } else {
    lb = lb0;
    ub = ub0;
  }
  // a phase boundary: bound reads of the next phase are not merged with this one's
  auto phase = [&]() __attribute__((always_inline)) {
    if constexpr (kBndLds) {
      lb.relaunder();
      ub.relaunder();
    }
  };
  // two group tests at once: ballots in a wave, one exchange for groups wider than a wave
  auto group_tests2 = [&](bool c0_, bool c1_, bool& r0, bool& r1) __attribute__((always_inline)) {
    if constexpr (G > 64) {
      double t[2] = {c0_ ? 1.0 : 0.0, c1_ ? 1.0 : 0.0};
      greduce_n<G, 3, 3>(t, xw);
      r0 = t[0] > 0.5;
      r1 = t[1] > 0.5;
    } else {
      r0 = gall<G, G * R>(c0_, xw);
      r1 = gall<G, G * R>(c1_, xw);
    }
  };
  const double nbound = gsum<G>((double)nbnd_l, xw);
  // ---- decoupled suffix (linear models; riccati.h DEC).  On stages k >= kb every table is
  //      decoupled (B = 0, no x-u Hessian block) and no state is bounded, so with delta = 0
  //      the stage Hessian's x block, A and P_{k+1} -- hence P_k -- are the same at every
  //      factorisation of a solve (fs is fixed after its first iteration).  Once a
  //      factorisation with delta = 0 stored P_k in Pk (pcv), the recursion reuses it there
  //      and only carries the vector part: the cart-pole QP's 95 move-blocked stages of
  //      100.  kb is set at every solve's first iteration (the tables may change per step).
  constexpr bool kDec = DecSuffixOf<Model>::value;
  bool xfree = true;
#pragma unroll
  for (int i = 0; i < NX; ++i) xfree = xfree && !hL[i] && !hU[i];
  int kb = N + 1;
  bool pcv = false;
  // the cross-launch cache was invalid at this solve's start (a cold handle, new tables): only
  // such a solve publishes, so a launch that found a valid cache never rewrites its header while
  // other groups may still be reading it (a group recovering from an inertia correction computes
  // the suffix afresh but does not publish)
  bool pc_miss = false;
  // the cross-launch cache of the suffix's P_k applies to shared tables at fs = 1 only
  auto pcache_ok = [&](double fs_) __attribute__((always_inline)) {
    return kDec && a.pcache != nullptr && fs_ == 1.0 && !a.lin.per_instance && a.tabseq == nullptr;
  };

  // ---- initial point
  double z[NZ];
#pragma unroll
  for (int i = 0; i < NZ; ++i) z[i] = 0.0;
  if (hasX) {
    if (a.w0) {
      const double* w0 = a.w0 + (size_t)inst * nw;
      for (int i = 0; i < NX; ++i) z[i] = w0[ixw<NX, NU>(k, i)];
      if (hasU)
        for (int i = 0; i < NU; ++i) z[NX + i] = w0[iuw<NX, NU>(k, i)];
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i) z[i] = x0[i];  // repmat(state_init), U = 0
    }
  }
  // bound push (IPOPT bound_push / bound_frac = 1e-2; warm start: warm_start_bound_push)
  bool warm = a.warm != 0;
  double lx0[NZ];  // given bound multipliers (zU - zL) of my variables
#pragma unroll
  for (int i = 0; i < NZ; ++i) lx0[i] = 0.0;
  if (warm && a.lamx0 && hasX) {
    const double* l = a.lamx0 + (size_t)inst * nw;
    if (k > 0)
      for (int i = 0; i < NX; ++i) lx0[i] = l[ixw<NX, NU>(k, i)];
    if (hasU)
      for (int i = 0; i < NU; ++i) lx0[NX + i] = l[iuw<NX, NU>(k, i)];
  }
  double zL[NZ], zU[NZ];
  // starting point of one solve from z (primal guess) and lx0 (given zU - zL): IPOPT's
  // bound push and dual initialisation -- shared by the launch start and the warm restarts
  // of multi-step launches, so both give the same bits
  auto init_point = [&]() __attribute__((always_inline)) {
    const double push = warm ? a.bound_push : kBoundPush, frac = warm ? a.bound_push : kBoundFrac;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      if (hL[i] && hU[i]) {
        const double pl = fmin(push * fmax(1.0, fabs(lb[i])), frac * (ub[i] - lb[i]));
        const double pu = fmin(push * fmax(1.0, fabs(ub[i])), frac * (ub[i] - lb[i]));
        z[i] = fmin(fmax(z[i], lb[i] + pl), ub[i] - pu);
      } else if (hL[i]) {
        z[i] = fmax(z[i], lb[i] + push * fmax(1.0, fabs(lb[i])));
      } else if (hU[i]) {
        z[i] = fmin(z[i], ub[i] - push * fmax(1.0, fabs(ub[i])));
      }
      zL[i] = hL[i] ? (warm ? fmax(-lx0[i], a.mult_push) : 1.0) : 0.0;
      zU[i] = hU[i] ? (warm ? fmax(lx0[i], a.mult_push) : 1.0) : 0.0;
    }
  };
  init_point();
  double lam[NX];  // lambda_k: multiplier of g_k (the constraint defining X_k)
#pragma unroll
  for (int i = 0; i < NX; ++i) lam[i] = (warm && a.lam0 && hasX) ? a.lam0[(size_t)inst * ng + NX * k + i] : 0.0;

  // ---- stage evaluation (all lanes evaluate -- SIMD, no extra cost -- lanes without an
  //      interval mask the results; A and B keep their structural constants)
  //      Interval 0 integrates from the parameter x0, not from X_0 (the script's
  //      Xk = P[:n_states], F(x0=vertcat(Xk, P[3:]), p=U_0): multiple_shooting_casadi.py:125,157),
  //      so the lifted X_0 enters only g_0 = x0 - X_0: lane 0's A_0, its x-gradient and its x
  //      Hessian blocks are zero in the NLP.  Lane 0 evaluates at (x0, U_0), its x-gradient is
  //      masked here, and the Newton step treats A_0 as zero (K_0 = 0, P_0 = Sigma_x + delta,
  //      p_0 = the barrier gradient, dx_1 independent of dx_0: riccati / forward below).
  double xf[NX], qv, A[NX * NX], Bm[NX * NU], gq[NZ], Hs[NH];
  double cdef[NX], c0[NX];  // cdef = F(X_k,U_k) - X_{k+1} (constraint k+1), c0 = x0 - X_0 (lane 0)
  double fs = 1.0;
  // the stage's evaluation point: (x0, U_0) on lane 0, (X_k, U_k) elsewhere
  auto stage_point = [&](const double* zz, double* ze) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NX; ++i) ze[i] = (k == 0) ? x0[i] : zz[i];
#pragma unroll
    for (int i = 0; i < NU; ++i) ze[NX + i] = zz[NX + i];
  };
  // evaluation at the point (zz, ll): also the line search's first trial when the model's
  // kEvalInSearch is set
  auto eval_at = [&](const double* zz, const double* ll) __attribute__((always_inline)) {
    double ln[NX], xn[NX], own[2 * NX], nxt[2 * NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      own[i] = ll[i];
      own[NX + i] = zz[i];
    }
    group_next<G, 2 * NX>(own, nxt, xw);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      ln[i] = nxt[i];
      xn[i] = nxt[NX + i];
    }
    double ze[NZ];
    stage_point(zz, ze);
    if constexpr (R > 1)  // the replicas split the evaluation's sequential RK4 substeps
      Model::derivs_rep(ma, ctx, ze, ln, fs, xf, qv, A, Bm, gq, Hs, rho);
    else
      stage_derivs<Model, G>(ma, ctx, ze, ln, fs, xf, qv, A, Bm, gq, Hs);
    const double m = hasU ? 1.0 : 0.0, mx = (hasU && k > 0) ? 1.0 : 0.0;  // no x-gradient at X_0
    qv *= m;
    if constexpr (!Model::kTableHess)
#pragma unroll
      for (int i = 0; i < NH; ++i) Hs[i] *= m;
#pragma unroll
    for (int i = 0; i < NZ; ++i) gq[i] *= (i < NX) ? mx : m;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      cdef[i] = hasU ? xf[i] - xn[i] : 0.0;
      c0[i] = (valid && k == 0) ? x0[i] - zz[i] : 0.0;
    }
  };
  // fresh: xf .. c0 hold the evaluation at the current (z, lam) (group-uniform)
  bool fresh = false;
  // lz_ok: Lz holds this lane's barrier log-sum at the current z -- the line search's first trial
  // point, accepted as it stands (the update's z is that trial's zt bit for bit), so the next
  // iteration's barrier objective needs no second evaluation of the same logarithms
  bool lz_ok = false;
  double Lz = 0.0;
  auto sweep = [&]() __attribute__((always_inline)) {
    eval_at(z, lam);
    fresh = true;
  };

  double mu = warm ? a.mu_init : 0.1, tau = fmax(kTauMin, 1.0 - mu);
  const double mu_min = a.tol / 10.0;
  double theta_max = 0.0, theta_min = 0.0;  // set at the first iterate
  double dw_last = 0.0;
  __shared__ double fbuf[FilterLds<G>::kDoubles];  // the instances' filters (FilterLds)
  FilterLds<G> filt;
  filt.init(fbuf + threadIdx.x);
  // IPOPT's filter-reset heuristic: iterations in a row whose last rejected trial point was
  // rejected by the filter alone, and resets so far in this solve
  int frej = 0, nfreset = 0;
  // IPOPT termination: acceptable iterates in a row, scaled objective of the previous iterate
  // (acceptable_obj_change_tol); a tiny step forces the next barrier decrease
  int acc_count = 0;
  double f_last = -1e50;
  bool tiny_flag = false;
  // IPOPT's soft restoration and restoration phase (models with one: resto.h, out of line; the
  // iterate travels through the workspace a.ws).  In the soft phase the soft step replaces the
  // line search.
  constexpr bool kRes = RestoOf<Model>::value;
  const bool res_on = kRes && a.restoration != 0;  // kernel-uniform
  // The solve launch clears every thread's park slot first, so the resume launch that follows
  // sees exactly the instances THIS launch parked: the workspace is laid out by this launch's
  // thread count, and an earlier launch at another batch size may have left slots set there
  if constexpr (kRes && !RESUME)
    if (a.ws) a.ws[(long)(RestoWs::SC(NX, NZ) + RestoWs::sPEND) * a.ws_stride + gid] = 0.0;
  // Models whose line search evaluates derivatives at its first trial (the unicycle) take IPOPT's
  // soft restoration step in the solve loop (a cold block after the line search).  Only the
  // restoration phase proper parks the instance for the resume launch, so an instance whose line
  // search fails once does not serialise the rest of a multi-step launch.
  constexpr bool kSoftInline = kRes && Model::kEvalInSearch && !Model::kSOC;
  bool soft_tried = false;  // this iteration's soft trial failed (the resume launch skips it)
  bool soft = false;
  int soft_count = 0;
  bool parked = false;       // left to the resume launch at a failed line search (solve launch)
  bool pending_rec = false;  // resume launch: recover at the top of the next pass
  bool active = true;        // resume launch: this group is one the solve launch parked
  bool scaled = false;       // the solve's objective scaling is set (its first pass ran)
  int status = valid ? 2 : 0;
  bool done = !valid;
  int it = 0;        // iteration of this instance's current solve
  int its = 0;       // its iteration count when it finished
  const int K = a.steps > 1 ? a.steps : 1;
  int step = valid ? 0 : K - 1;  // closed-loop step of this instance (multi-step launches)
  // every per-lane array is defined on every lane (lanes past node N included): no
  // indeterminate values for the optimiser to exploit
  double dz[NZ] = {}, dlam[NX] = {}, dzL[NZ] = {}, dzU[NZ] = {};
  double Pk[NP] = {}, pk[NX] = {}, Kk[NU * NX] = {}, kfk[NU] = {};

#ifdef MPCX_STAMPS
  // 0 regularised iterations, 1 extra factorisations, 2 backtracks, 3 barrier updates,
  // 4 fraction-to-boundary-limited steps (alpha_max < 1), 5 tiny steps, 6 filter rejections,
  // 7 f-type (Armijo) acceptances, 8 factorisations by the sequential fallback of the scan,
  // 9 filter resets, 10 first trials rejected with increased infeasibility (SOC-eligible),
  // 11 accepted second-order corrections, 12 recoveries (soft restoration / restoration phase
  // calls, resto.h), 13 restoration-phase iterations, 14 filter additions that found all G
  // slots holding mutually non-dominated entries (filter_add; an entry was overwritten)
  int diag[kDiag] = {};
  unsigned long long st_acc[kStampSlots] = {};
  unsigned long long st_last = 0;
  int st_ph = 9;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
  // ---- multi-step launches: the closed-loop step boundary of an instance that finished a
  //      non-final step -- record it, plant x0 <- F(x0, u0*) on lane 0, shift primal and
  //      multipliers one node (Casadi/multiple_shooting_casadi.py:271-287, the same values
  //      the fused epilogue below writes), load the next step's references and schedule,
  //      and restart the solve exactly as a new launch would from those buffers.
  auto step_boundary = [&]() __attribute__((always_inline)) {
    const bool bnd = done && !parked && step < K - 1;  // group-uniform
    if (!__any(bnd)) return;
    constexpr int NS = NZ + NX + NZ;
    double own[NS], nxt[NS];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      own[i] = z[i];
      own[NZ + NX + i] = (zU[i] - zL[i]) / fs;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) own[NZ + i] = lam[i] / fs;
    group_next<G, NS>(own, nxt, xw);
    if (bnd) {
      if (k == 0 && valid) {  // lanes past the batch are done from the start: no status row of theirs
        if (a.status && rho == 0) a.status[(size_t)step * a.B + inst] = status;
        if (a.iters && rho == 0) a.iters[(size_t)step * a.B + inst] = its;
        double zp[NZ], xfp[NX], qp;
#pragma unroll
        for (int i = 0; i < NX; ++i) zp[i] = x0[i];
#pragma unroll
        for (int i = 0; i < NU; ++i) zp[NX + i] = z[NX + i];
        Model::value(ma, ctx, zp, xfp, qp);
#pragma unroll
        for (int i = 0; i < NX; ++i) x0[i] = xfp[i];
      }
      ++step;
      const int ivi = valid ? inst : 0;  // never index past the batch
      const double* Pn = a.Pseq ? a.Pseq + ((size_t)step * a.B + ivi) * a.p_stride : Pin;
      ModelArgs mst = ma;
      if (a.tabseq) {
        mst.lin.tab = a.tabseq + (size_t)step * a.B * N;
        mst.lin.per_instance = 1;
      }
      Model::load_ctx(mst, ivi, Pn, k, hasU, ctx);
      const bool lastX = (k == N), lastU = (k == N - 1);
      warm = a.warm_next != 0;
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        z[i] = hasX ? (lastX ? own[i] : nxt[i]) : 0.0;
        lam[i] = (warm && hasX) ? (lastX ? own[NZ + i] : nxt[NZ + i]) : 0.0;
        lx0[i] = (warm && hasX && k > 0) ? (lastX ? own[NZ + NX + i] : nxt[NZ + NX + i]) : 0.0;
      }
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        z[NX + i] = hasU ? (lastU ? own[NX + i] : nxt[NX + i]) : 0.0;
        lx0[NX + i] = (warm && hasU) ? (lastU ? own[NZ + 2 * NX + i] : nxt[NZ + 2 * NX + i]) : 0.0;
      }
      init_point();
      fresh = false;
      lz_ok = false;
      mu = warm ? a.mu_init : 0.1;
      tau = fmax(kTauMin, 1.0 - mu);
      fs = 1.0;
      theta_max = theta_min = 0.0;
      dw_last = 0.0;
      filt.clear();
      frej = nfreset = 0;
      acc_count = 0;
      f_last = -1e50;
      tiny_flag = false;
      soft = false;
      soft_count = 0;
      scaled = false;
      status = 2;
      done = false;
      it = 0;
      its = 0;
    }
  };

  // every pass is one IPM iteration for the instances still solving; instances that
  // finished a step of a multi-step launch restart at the top of the next pass.  Bounded:
  // each step ends after at most max_iter + 1 passes.
  // ---- resume launch: only the groups the solve launch parked run, from their saved state
  if constexpr (RESUME) {
    double* const wsl = a.ws + gid;
    const long wst = a.ws_stride;
    auto W = [&](int i) __attribute__((always_inline)) -> double& { return wsl[(long)i * wst]; };
    constexpr int S = RestoWs::SC(NX, NZ);
    active = valid && W(S + RestoWs::sPEND) != 0.0;
    if (!__any(active)) return;  // wave-uniform (a multi-wave group's waves agree)
    if (active) {
      W(S + RestoWs::sPEND) = 0.0;
#ifdef MPCX_STAMPS
      if (g_mpcx_diag)
        for (int i = 0; i < kDiag; ++i) diag[i] = g_mpcx_diag[(size_t)inst * kDiag + i];
#endif
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        z[i] = W(RestoWs::XZ + i);
        zL[i] = W(RestoWs::XZL(NX, NZ) + i);
        zU[i] = W(RestoWs::XZU(NX, NZ) + i);
      }
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        lam[i] = W(RestoWs::XL(NZ) + i);
        x0[i] = W(RestoWs::XX0(NX, NZ) + i);
      }
      fs = W(S + RestoWs::sFS);
      mu = W(S + RestoWs::sMU);
      tau = W(S + RestoWs::sTAU);
      theta_max = W(S + RestoWs::sTHMAX);
      theta_min = W(S + RestoWs::sTHMIN);
      dw_last = W(S + RestoWs::sDWLAST);
#pragma unroll
      for (int j = 0; j < FilterLds<G>::S; ++j) {
        filt.th(j) = W(S + RestoWs::sFTH + j);
        filt.ph(j) = W(S + RestoWs::sFPH + j);
      }
      filt.next = (int)W(S + RestoWs::sFNEXT);
      filt.n = (int)W(S + RestoWs::sFN);
      frej = (int)W(S + RestoWs::sFREJ);
      nfreset = (int)W(S + RestoWs::sNFRESET);
      acc_count = (int)W(S + RestoWs::sACC);
      f_last = W(S + RestoWs::sFLAST);
      soft = W(S + RestoWs::sSOFT) != 0.0;
      soft_count = (int)W(S + RestoWs::sSOFTN);
      it = (int)W(S + RestoWs::sIT);
      step = (int)W(S + RestoWs::sSTEP);
      warm = W(S + RestoWs::sWARM) != 0.0;
      if (a.Pseq && step > 0) {  // the step's references (multi-step launches)
        const double* Pn = a.Pseq + ((size_t)step * a.B + inst) * a.p_stride;
        Model::load_ctx(ma, inst, Pn, k, hasU, ctx);
      }
      scaled = true;
      pending_rec = true;
    } else {
      done = true;
      step = K - 1;
    }
  }
  const long max_pass = (long)K * (a.max_iter + 2);
  for (long pass = 0; pass <= max_pass; ++pass, ++it) {
    if (K > 1) step_boundary();
    if constexpr (RESUME) {
      // soft restoration / restoration phase from the state saved at the failed line search
      // (resto.h); the pass then goes on at the recovered point
      if (MPCX_COLD(__any(pending_rec))) {
        if (pending_rec) {
          pending_rec = false;
          double* wsl = a.ws + gid;
          long wst = a.ws_stride;
          asm volatile("" : "+v"(wsl), "+v"(wst));  // no workspace addresses hoisted out of the loop
          auto W = [&](int i) __attribute__((always_inline)) -> double& { return wsl[(long)i * wst]; };
          constexpr int S = RestoWs::SC(NX, NZ);
          RecIO io;
          io.it = (int)W(S + RestoWs::sIT);
          io.max_iter = a.max_iter;
          io.k = k;
          io.N = N;
          io.nw = nw;
          io.ng = ng;
          io.valid = valid;
          io.hasX = hasX;
          io.hasU = hasU;
          io.acc_now = W(S + RestoWs::sACCNOW) != 0.0;
          io.soft_tried = W(S + RestoWs::sSOFTTRIED) != 0.0;
          io.tol = a.tol;
          io.mu_min = mu_min;
          io.fs = fs;
          io.nbound = nbound;
          io.thk = W(S + RestoWs::sTHK);
          io.phk = W(S + RestoWs::sPHK);
          io.gd = W(S + RestoWs::sGD);
          io.amax = W(S + RestoWs::sAMAX);
          io.az = W(S + RestoWs::sAZ);
          io.sw_a = W(S + RestoWs::sSWA);
          io.mu = mu;
          io.tau = tau;
          io.theta_max = theta_max;
          io.theta_min = theta_min;
          io.dw_last = dw_last;
          io.frej = frej;
          io.nfreset = nfreset;
          io.soft = soft;
          io.soft_count = soft_count;
          io.xslot = xw.slot;
          io.fovf = 0;
          recover<Model, G>(io, filt, ma, ctx, wsl, wst, a.lbw, a.ubw, xch);
#pragma unroll
          for (int i = 0; i < NZ; ++i) {
            z[i] = W(RestoWs::XZ + i);
            zL[i] = W(RestoWs::XZL(NX, NZ) + i);
            zU[i] = W(RestoWs::XZU(NX, NZ) + i);
          }
#pragma unroll
          for (int i = 0; i < NX; ++i) lam[i] = W(RestoWs::XL(NZ) + i);
          mu = io.mu;
          tau = io.tau;
          theta_max = io.theta_max;
          theta_min = io.theta_min;
          dw_last = io.dw_last;
          frej = io.frej;
          nfreset = io.nfreset;
          soft = io.soft;
          soft_count = io.soft_count;
          xw.slot = io.xslot;
          if (io.reset_acc) acc_count = 0;
          tiny_flag = false;
#ifdef MPCX_STAMPS
          if (io.it_next > io.it + 1) diag[13] += io.it_next - io.it - 1;  // restoration iterations
          diag[14] += io.fovf;
#endif
          if (io.status >= 0) {
            done = true;
            status = io.status;
            its = io.its;
          }
          it = io.it_next;  // this pass is that iteration
        }
      }
    }
    // ------------------------------------------------------------ evaluation
    //  skipped when the line search already evaluated the accepted point; only the groups
    //  that need it evaluate (exec-masked, group-uniform), so an instance's sequence of
    //  evaluation sites -- and its bits -- never depends on its wave neighbours
    //  (models without kEvalInSearch evaluate unconditionally: nothing then stays live
    //  across the back-edge)
    if constexpr (Model::kEvalInSearch) {
      if (__any(!fresh && !done))
        if (!fresh) sweep();
    } else {
      sweep();
    }
    if (!scaled) {
      scaled = true;
      // objective scaling (IPOPT nlp_scaling_method = gradient-based, max_gradient = 100).
      // With lambda scaled by the same factor the Lagrangian's gradient and Hessian scale
      // exactly by fs, so no re-evaluation is needed.
      double gm = 0;
#pragma unroll
      for (int i = 0; i < NZ; ++i) gm = fmax(gm, fabs(gq[i]));
#ifdef MPCX_DEBUG_PRINT
      const double gm_local = gm;
#endif
      gm = gmax<G>(gm, xw);
#ifdef MPCX_DEBUG_PRINT
      if (inst == 0 && (k % 32) == 0)
        printf("k=%d wave=%d gm_local=%g gm=%g slot=%d nbound=%g lds=%p\n", k, (int)(threadIdx.x >> 6), gm_local, gm,
               xw.slot, nbound, (void*)xw.buf);
#endif
      fs = gm > 100.0 ? 100.0 / gm : 1.0;
      if constexpr (kDec) {
        const bool d = !hasX || (xfree && (k == N || ctx.dec));
        kb = (int)gmax<G>(d ? -1.0 : (double)k, xw) + 1;
        pcv = false;
        pc_miss = false;
        // the suffix's P_k as an earlier launch of these tables computed them at fs = 1 and
        // delta = 0 (from identical operands: the same bits this solve's first factorisation
        // would produce), so even the first factorisation takes the reused path
        if (pcache_ok(fs)) {
          const double* hdr = a.pcache + (size_t)(N + 1) * NP;
          if (hdr[0] > 0.0 && hdr[0] < a.pc_epoch && hdr[1] == a.pc_gen && hdr[2] == (double)kb) {
            if (k >= kb && k <= N)
#pragma unroll
              for (int i = 0; i < NP; ++i) Pk[i] = a.pcache[(size_t)k * NP + i];
            pcv = true;
          } else {
            pc_miss = true;
          }
        }
      }
      if (fs != 1.0) {  // group-uniform; given multipliers belong to the unscaled problem
#pragma unroll
        for (int i = 0; i < NX; ++i) lam[i] *= fs;
#pragma unroll
        for (int i = 0; i < NZ; ++i) gq[i] *= fs;
        if constexpr (!Model::kTableHess)
#pragma unroll
          for (int i = 0; i < NH; ++i) Hs[i] *= fs;
        if (warm)
#pragma unroll
          for (int i = 0; i < NZ; ++i) {
            if (hL[i]) zL[i] = fmax(zL[i] * fs, a.mult_push);
            if (hU[i]) zU[i] = fmax(zU[i] * fs, a.mult_push);
          }
      }
      double theta0 = 0;
#pragma unroll
      for (int i = 0; i < NX; ++i) theta0 += fabs(cdef[i]) + fabs(c0[i]);
      theta0 = gsum<G>(theta0, xw);
      theta_max = 1e4 * fmax(1.0, theta0);
      theta_min = 1e-4 * fmax(1.0, theta0);
    }
    STAMP(0);
    phase();
    // ------------------------------------------------------------ optimality error
    double ln[NX];
    group_next<G, NX>(lam, ln, xw);
    double Ed = 0, Ecomp0 = 0, Ec = 0, lam1 = 0, z1 = 0;
    double rd[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) rd[i] = 0;
    if (hasX) {
#pragma unroll
      for (int i = 0; i < NX; ++i) rd[i] = gq[i] - lam[i];
      if (hasU) {
        if (k > 0)  // (X_0 enters only g_0)
#pragma unroll
          for (int j = 0; j < NX; ++j)
#pragma unroll
            for (int m = 0; m < NX; ++m)
              if (Model::AMASK & (1ull << (m * NX + j))) rd[j] = fma(Model::jacA(ctx, A)[m * NX + j], ln[m], rd[j]);
#pragma unroll
        for (int l = 0; l < NU; ++l) {
          double acc = gq[NX + l];
#pragma unroll
          for (int m = 0; m < NX; ++m)
            if (Model::BMASK & (1ull << (m * NU + l))) acc = fma(Model::jacB(ctx, Bm)[m * NU + l], ln[m], acc);
          rd[NX + l] = acc;
        }
      }
#pragma unroll
      for (int i = 0; i < NX; ++i) lam1 += fabs(lam[i]);
    }
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      rd[i] += zU[i] - zL[i];
      Ed = qmax_abs(Ed, rd[i]);
      z1 += zL[i] + zU[i];
      // branchless (the asm max cannot be speculated; max(E, 0) = E for E >= 0)
      Ecomp0 = qmax_abs(Ecomp0, hL[i] ? (z[i] - lb[i]) * zL[i] : 0.0);
      Ecomp0 = qmax_abs(Ecomp0, hU[i] ? (ub[i] - z[i]) * zU[i] : 0.0);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) Ec = qmax_abs(qmax_abs(Ec, cdef[i]), c0[i]);
    // Ed, Ec, Ecomp0 stay per lane: every test below is a threshold on their group maximum, which
    // holds iff it holds on every lane (gall: one ballot instead of a max reduction each; max is
    // exact and the division by a positive group-uniform scaling monotone, so the decisions are the
    // ones the reduced values give)
    double sums[3] = {lam1, z1, hasU ? qv : 0.0};  // one exchange for the three group sums
    STAMP_SUB(14);
    greduce_n<G, 0, 0, 0>(sums, xw);
    STAMP_SUB(15);
    lam1 = sums[0];
    z1 = sums[1];
    // IPOPT's scalings s_d = max(s_max, (|lam|_1 + |z|_1) / (m + n)) / s_max and s_c = max(s_max,
    // |z|_1 / n_b) / s_max are exactly 1 unless the sum exceeds s_max times the count (a rounded
    // quotient that reaches s_max from above still gives 1): the IEEE divisions -- group-uniform
    // ~12-instruction sequences -- only run on waves where some instance needs them
    const bool sd1 = !(lam1 + z1 > kSmax * (double)(ng + nw));
    const bool sc1 = !(nbound > 0 && z1 > kSmax * nbound);
    double sd = 1.0, sc = 1.0, Eds = Ed, Ecs = Ecomp0;  // Ed / s_d, Ecomp0 / s_c (this lane's)
    if (__any(!sd1 || !sc1)) {
      if (!sd1) {
        sd = fmax(kSmax, (lam1 + z1) / (double)(ng + nw)) / kSmax;
        Eds = Ed / sd;
      }
      if (!sc1) {
        sc = fmax(kSmax, z1 / nbound) / kSmax;
        Ecs = Ecomp0 / sc;
      }
    }
    const double E0 = fmax(fmax(Eds, Ec), Ecs);  // this lane's part of the scaled NLP error
    // IPOPT OptimalityErrorConvergenceCheck: tol with the unscaled dual infeasibility,
    // constraint violation and complementarity tests; then the acceptable level (all of
    // acceptable_* and the objective change from the previous iterate) for acceptable_iter
    // iterates in a row.  fcur = the scaled objective.
    const double fcur = fs * sums[2];
    bool conv_g, acc_g;
    group_tests2(E0 <= a.tol && Ed <= a.dual_inf_tol * fs && Ec <= a.constr_viol_tol && Ecomp0 <= a.compl_inf_tol * fs,
                 E0 <= a.acc_tol && Ed <= a.acc_dual_inf_tol * fs && Ec <= a.acc_constr_viol_tol &&
                     Ecomp0 <= a.acc_compl_inf_tol * fs,
                 conv_g, acc_g);
    const bool acceptable_now = acc_g && fabs(fcur - f_last) <= a.acc_obj_change_tol * fmax(1.0, fabs(fcur));
    if (conv_g && !done) {
      done = true;
      status = 0;
      its = it;
    }
    if (!done) {
      f_last = fcur;
      acc_count = (a.acc_iter > 0 && acceptable_now) ? acc_count + 1 : 0;
      if (a.acc_iter > 0 && acc_count >= a.acc_iter) {
        done = true;
        status = 1;
        its = it;
      }
    }
    if (!done && it >= a.max_iter) {
      done = true;
      status = 2;
      its = a.max_iter;
    }
#ifdef MPCX_DEBUG_PRINT
    {
      const double Edg = gmax<G>(Ed, xw), Ecg = gmax<G>(Ec, xw), E0g = gmax<G>(E0, xw);
      if (inst == 0 && (k % 64) == 0)
        printf("OPT it=%d k=%d fs=%g Ed=%g Ec=%g E0=%g sd=%g lam1=%g z1=%g\n", it, k, fs, Edg, Ecg, E0g, sd, lam1, z1);
    }
#endif
    if (__all((done && step == K - 1) || parked)) break;
    // multi-step launches: a wave whose instances all just finished a step skips the rest of
    // this pass (its Newton step would be discarded) and restarts at the step boundary
    if (K > 1 && __all(done)) continue;

    STAMP(1);
    phase();
    // ------------------------------------------------------------ barrier update
    // (IPOPT monotone update with mu_allow_fast_monotone_decrease: repeated while the barrier
    //  test holds; a tiny step forces the first decrease)
    for (int rep = 0; rep < 32; ++rep) {
      double Ecm = 0;
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        Ecm = qmax_abs(Ecm, hL[i] ? (z[i] - lb[i]) * zL[i] - mu : 0.0);
        Ecm = qmax_abs(Ecm, hU[i] ? (ub[i] - z[i]) * zU[i] - mu : 0.0);
      }
      double Ecms = Ecm;  // Ecm / s_c (this lane's; the test is a group threshold test, as above)
      if (__any(!sc1))
        if (!sc1) Ecms = Ecm / sc;
      const double Emu = fmax(fmax(Eds, Ec), Ecms);
      const bool dec = !done && (gall<G, G * R>(Emu <= kKappaEps * mu, xw) || (tiny_flag && rep == 0)) && mu > mu_min;
      if (dec && !done) DIAG(3);
      if (dec) {
        static_assert(kThetaMu == 1.5, "mu^theta_mu evaluated as mu * sqrt(mu)");
        mu = fmax(mu_min, fmin(kKappaMu * mu, mu * sqrt(mu)));
        tau = fmax(kTauMin, 1.0 - mu);
        filt.clear();
      }
      if (!__any(dec)) break;
    }
    tiny_flag = false;
    STAMP(2);
    phase();
    // ------------------------------------------------------------ barrier gradient, Sigma
    double sig[NZ], gp[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      sig[i] = 0;
      gp[i] = gq[i];
      // one rcp64 per slack instead of IEEE divisions (each a ~10-instruction sequence)
      if (hL[i]) {
        const double rs = rcp64(z[i] - lb[i]);
        sig[i] = fma(zL[i], rs, sig[i]);
        gp[i] = fma(-mu, rs, gp[i]);
      }
      if (hU[i]) {
        const double rs = rcp64(ub[i] - z[i]);
        sig[i] = fma(zU[i], rs, sig[i]);
        gp[i] = fma(mu, rs, gp[i]);
      }
    }

    STAMP(3);
    phase();
    // ------------------------------------------------------------ Riccati + inertia correction
    // Models with a workspace chain stash (kernels.h WsStashOf: the 6-state bicycle) keep the
    // stage Hessian and Sigma in the workspace instead of registers across the inertia-correction
    // loop: every attempt re-reads them (node-parallel, coalesced), so neither is live across the
    // sequential chain, whose operands then fit the registers (no scratch round trip per step)
    if constexpr (kWsStash) {
      double* r = const_cast<double*>(wsrec());
#pragma unroll
      for (int i = 0; i < NH; ++i) r[kRH + i] = Hs[i];
#pragma unroll
      for (int i = 0; i < NZ; ++i) r[kRS + i] = sig[i];
#pragma unroll
      for (int i = 0; i < NX * NX; ++i) r[kRA + i] = (Model::AMASK & (1ull << i)) ? A[i] : 0.0;
#pragma unroll
      for (int i = 0; i < NX * NU; ++i) r[kRB + i] = (Model::BMASK & (1ull << i)) ? Bm[i] : 0.0;
    }
    // this lane's Jacobians back from the workspace (kWsStash), for the phases after the chain
    auto ws_jac = [&](double* Aw, double* Bw) __attribute__((always_inline)) {
      const double* r = wsrec();
#pragma unroll
      for (int i = 0; i < NX * NX; ++i) Aw[i] = (Model::AMASK & (1ull << i)) ? wsload(r, kRA + i) : 0.0;
#pragma unroll
      for (int i = 0; i < NX * NU; ++i) Bw[i] = (Model::BMASK & (1ull << i)) ? wsload(r, kRB + i) : 0.0;
    };
    double delta = 0.0;
    bool need = !done;  // instance still needs a factorisation
    bool failed = false;
    bool first = true;
    Fac<NX, NU> fac = {};
    // decoupled suffix: this factorisation starts without stored suffix value functions
    const bool fresh_fac = !pcv;
    for (int attempt = 0; attempt < 64; ++attempt) {
      if (!__any(need)) break;
      STAMP_SUB(10);
      // node-parallel: stage Hessian + Sigma + delta (off the sequential path)
      double Hd[NH], sgv[NZ];
      // stage Hessian (table-Hessian models: 2 fs W of the stage table; none at node N)
      const double hsc = Model::kTableHess ? (hasU ? 2.0 * fs : 0.0) : 1.0;
      const double* Aop = Model::jacA(ctx, A);
      const double* Bop = Model::jacB(ctx, Bm);
      if constexpr (kWsStash) {
        const double* r = wsrec();
#pragma unroll
        for (int i = 0; i < NH; ++i) Hd[i] = wsload(r, kRH + i);
#pragma unroll
        for (int i = 0; i < NZ; ++i) sgv[i] = wsload(r, kRS + i);
      } else {
        const double* Hsrc = Model::hessW(ctx, Hs);
#pragma unroll
        for (int i = 0; i < NH; ++i) Hd[i] = Model::kTableHess ? hsc * Hsrc[i] : Hsrc[i];
#pragma unroll
        for (int i = 0; i < NZ; ++i) sgv[i] = sig[i];
      }
#pragma unroll
      for (int i = 0; i < NZ; ++i) Hd[symix(i, i, NZ)] += sgv[i] + delta;

      // backward sweep: node N .. 0 (value function moves lane k+1 -> k)
      double P[NP], p[NX];
      bool okl = true;
      bool seq = true;  // group-uniform: this instance needs the sequential recursion
      if constexpr (Model::kParallelRiccati) {
        // ---- log-depth associative scan of conditional value functions (pscan.h)
        RElem<NX> e;
        bool eok = true;
        if (hasU) {
          eok = relem_stage<NX, NU, Model::AMASK, Model::BMASK>(Hd, gp, Aop, Bop, cdef, e);
        } else {
          relem_identity<NX>(e);
          if (hasX) {  // node N: terminal (0, 0, 0, Sigma_x + delta, barrier gradient)
#pragma unroll
            for (int i = 0; i < NX * NX; ++i) e.A[i] = 0.0;
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
              for (int j = i; j < NX; ++j) e.J[symix(i, j, NX)] = (i == j) ? sgv[i] + delta : 0.0;
              e.p[i] = gp[i];
            }
          }
        }
        // Hillis-Steele suffix scan over the whole group through the LDS buffer `sbuf`
        // (partner = thread t + d; block-uniform trip count, two barriers per level)
        const int t = (int)threadIdx.x;
        for (int d = 1; d < G && d <= N; d <<= 1) {
          relem_store<NX>(e, sbuf, kSBS, t);
          __syncthreads();
          if (k + d < G) relem_combine_lds<NX>(e, sbuf + t + d, kSBS);
          __syncthreads();
        }
        // value function of node k+1, then ONE node-parallel Riccati step per lane: gains,
        // inertia test and (P_k, p_k) as the sequential recursion would produce them
        double Jn[NP + NX], nx_[NP + NX];
#pragma unroll
        for (int i = 0; i < NP; ++i) Jn[i] = e.J[i];
#pragma unroll
        for (int i = 0; i < NX; ++i) Jn[NP + i] = e.p[i];
        group_next<G, NP + NX>(Jn, nx_, xw);
        const double dl = (k == N) ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < NX; ++i) {
#pragma unroll
          for (int j = i; j < NX; ++j) P[symix(i, j, NX)] = (i == j) ? dl * (sgv[i] + delta) : 0.0;
          p[i] = dl * gp[i];
        }
        double dev = 0.0, mag = 1.0;
        if (hasU) {
          okl = riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, false, AOneOf<Model>::value>(Hd, gp, Aop, Bop, cdef, nx_,
                                                                                                 nx_ + NP, P, p, fac);
#pragma unroll
          for (int i = 0; i < NP; ++i) {
            dev = fmax(dev, fabs(P[i] - e.J[i]));
            mag = fmax(mag, fabs(P[i]));
          }
#pragma unroll
          for (int i = 0; i < NX; ++i) {
            dev = fmax(dev, fabs(p[i] - e.p[i]));
            mag = fmax(mag, fabs(p[i]));
          }
        }
        // scan usable: stage R positive definite, finite, and consistent with the step
        const bool good = eok && dev <= 1e-8 * mag;  // false for NaN
        seq = !gall<G, G * R>(good, xw);
        DIAG_IF(seq && !done, 8);
      }
      // Stash: the iterate, its bound multipliers, bounds and lam are live across the sequential
      // chain but unused in it; for the 6-state model they go to the LDS value cache (idle
      // between evaluations) so the chain's operands keep registers instead of scratch
      // (the 6-state row chain's ring occupies that cache: the iterate waits in the workspace record)
      constexpr bool kStash = !Model::kParallelRiccati && NX >= 6 && Model::kTrigSlots >= 5 * NZ + NX;
      auto stash = [&](bool back) __attribute__((always_inline)) {
        if constexpr (kStash) {
          double* t = kRow6 ? const_cast<double*>(wsrec()) + kRZ : tcache + threadIdx.x;
          constexpr int st = kRow6 ? 1 : kSBS;
          auto mv = [&](double& v, int o) __attribute__((always_inline)) {
            if (back) v = kRow6 ? wsload(t, o) : t[o * st];
            else t[o * st] = v;
          };
#pragma unroll
          for (int i = 0; i < NZ; ++i) {
            mv(z[i], i);
            mv(zL[i], NZ + i);
            mv(zU[i], 2 * NZ + i);
            mv(lb0[i], 3 * NZ + i);
            mv(ub0[i], 4 * NZ + i);
          }
#pragma unroll
          for (int i = 0; i < NX; ++i) mv(lam[i], 5 * NZ + i);
        }
      };
      stash(false);
      if (__any(seq)) {  // sequential recursion (models without the scan, or its fallback)
        if (seq && !kRow && !kRow6) {  // (the row chains set P, p after the chain: not live across it)
          okl = true;
          const double dl = (k == N) ? 1.0 : 0.0;  // P_N = Sigma_x + delta, p_N = barrier gradient
#pragma unroll
          for (int i = 0; i < NX; ++i) {
#pragma unroll
            for (int j = i; j < NX; ++j) P[symix(i, j, NX)] = (i == j) ? dl * (sgv[i] + delta) : 0.0;
            p[i] = dl * gp[i];
          }
        }
        // decoupled suffix: with P_{k+1} reused, s = P_{k+1} c + p_{k+1} needs only p on the
        // chain; P_{k+1} c comes from the stored Pk of node k+1, off the chain
        const bool reuse = kDec && pcv && delta == 0.0;  // group-uniform
        double vpc[kDec ? NX : 1];
        bool okd = true;
        if constexpr (kDec) {
          double Pn1[NP];
          group_next<G, NP>(Pk, Pn1, xw);
#pragma unroll
          for (int i = 0; i < NX; ++i) vpc[i] = riccati_pc_row<NX>(Pn1, cdef, i);
          // reused stages: factors and P_k set here, off the chain (dec_prefactor)
          if (reuse && k >= kb && k < N) {
            okd = dec_prefactor<NX, NU>(Hd, fac);
#pragma unroll
            for (int i = 0; i < NP; ++i) P[i] = Pk[i];
          }
        }
        // steps j >= jc are reused-suffix steps for every group of the wave: they run first, in
        // a loop of their own that moves only p (the same operations as the mixed loop's cheap
        // steps; A stays in the stage table: 25 more live registers here measured slower)
        int jc = N;
        if constexpr (kDec) {
          if (__all(reuse)) {
            XWave<64> xw1{nullptr, 0};
            jc = G >= 64 ? kb : (int)greduce<64, OpMax>((double)kb, xw1);  // max over the wave's groups
            jc = __builtin_amdgcn_readfirstlane(jc);  // wave-uniform: scalar loop bounds
          }
        }
        // The reused suffix as a log-depth scan (multi-wave groups: one instance per block).  On
        // a reused stage p_k = A^T p_{k+1} + r_k with r_k = gp_x + A^T (P_{k+1} c), and when every
        // stage of the suffix uses the same table (shared tables) the composition of d steps is
        // the uniform (A^T)^d: a radix-4 Hillis-Steele suffix scan
        //   v_k += (A^T)^d v_{k+d} + (A^T)^{2d} v_{k+2d} + (A^T)^{3d} v_{k+3d},   d = 1, 4, 16, 64
        // carries only the NX-vector through ping-pong LDS buffers, ONE barrier per level (config 5:
        // 4 levels replace the suffix's 95 dependent steps; a radix-2 scan needs 7 levels of two
        // barriers).  The powers (A^T)^(j 4^l) depend only on the table: they are formed by NX^2
        // threads in LDS the first time a launch scans a table and kept there for the launch.
        STAMP_SUB(11);
        bool sscan = false;  // group-uniform
        if constexpr (kDec && G > 64) {
          if (jc < N && !a.lin.per_instance && a.tabseq == nullptr) {
            const bool mine = k >= jc && k < N;
            const double ti = (double)((ctx.A - a.lin.A) / (NX * NX));  // my stage's table
            double tt[2] = {mine ? ti : -1.0, mine ? ti : 1e300};
            greduce_n<G, 1, 2>(tt, xw);
            const double tmax = tt[0];
            sscan = tt[1] == tmax;
            if (sscan) {
              double* mpow = dscan + 2 * NX * kSBS;  // (A^T)^(j 4^l) at mpow[(3 l + j - 1) NX^2], row-major
              const int t = (int)threadIdx.x;
              constexpr int kLev = G > 64 ? (G <= 256 ? 4 : 5) : 1;  // 4^kLev >= G
              if (tmax != pow_tab) {  // block-uniform
                const double* Au = a.lin.A + (size_t)tmax * NX * NX;
                auto mul = [&](int dst, int x, int y) __attribute__((always_inline)) {  // mpow[dst] = X Y
                  if (t < NX * NX) {
                    const double* X = mpow + x * NX * NX;
                    const double* Y = mpow + y * NX * NX;
                    const int i = t / NX, j = t % NX;
                    double acc = X[i * NX] * Y[j];
#pragma unroll
                    for (int m = 1; m < NX; ++m) acc = fma(X[i * NX + m], Y[m * NX + j], acc);
                    mpow[dst * NX * NX + t] = acc;
                  }
                  __syncthreads();
                };
                if (t < NX * NX) mpow[t] = Au[(t % NX) * NX + t / NX];
                __syncthreads();
                for (int l = 0; l < kLev; ++l) {
                  if (l > 0) mul(3 * l, 3 * l - 2, 3 * l - 2);  // (A^T)^(4^l) = ((A^T)^(2 4^(l-1)))^2
                  mul(3 * l + 1, 3 * l, 3 * l);                 // (A^T)^(2 4^l)
                  mul(3 * l + 2, 3 * l + 1, 3 * l);             // (A^T)^(3 4^l)
                }
                pow_tab = tmax;
              }
              double v[NX];
#pragma unroll
              for (int i = 0; i < NX; ++i) {
                double acc = gp[i];
#pragma unroll
                for (int m = 0; m < NX; ++m)
                  if (Model::AMASK & (1ull << (m * NX + i))) acc = fma(Aop[m * NX + i], vpc[m], acc);
                v[i] = mine ? acc : (k == N ? p[i] : 0.0);
              }
              double* buf = dscan;  // ping-pong: level l reads buf[l % 2], writes buf[(l + 1) % 2]
#pragma unroll
              for (int i = 0; i < NX; ++i) buf[i * kSBS + t] = v[i];
              __syncthreads();
              for (int l = 0, d = 1; l < kLev && d <= N; ++l, d *= 4) {
                const double* cur = dscan + (l & 1) * NX * kSBS;
                double* nxt = dscan + ((l + 1) & 1) * NX * kSBS;
#pragma unroll
                for (int q = 1; q <= 3; ++q) {
                  // the matrix spread over each 16-lane row (lane r: elements r and 16 + r) and
                  // applied by row-broadcast FMAs (collectives.h matvec_bcast): the block-uniform
                  // elements were 25 broadcast LDS reads, each a round trip on the FMA chain.  Every
                  // lane takes part (a broadcast source lane must be active); lanes without a
                  // partner keep v.
                  const double* M = mpow + (3 * l + q - 1) * NX * NX;
                  const int r = t & 15;
                  const double mA = M[min(r, NX * NX - 1)];  // (in bounds for NX * NX < 16 too)
                  const double mB = NX * NX > 16 ? M[16 + min(r, NX * NX - 17)] : 0.0;
                  const bool on = t + q * d < G;
                  const int src = on ? t + q * d : t;
                  double w[NX], acc[NX];
#pragma unroll
                  for (int i = 0; i < NX; ++i) {
                    w[i] = cur[i * kSBS + src];
                    acc[i] = v[i];
                  }
                  matvec_bcast<NX>(acc, w, mA, mB);
#pragma unroll
                  for (int i = 0; i < NX; ++i) v[i] = on ? acc[i] : v[i];
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) nxt[i * kSBS + t] = v[i];
                __syncthreads();
              }
              if (seq && mine) {
#pragma unroll
                for (int i = 0; i < NX; ++i) p[i] = v[i];
                fac.g0 = gp[NX];
                if constexpr (NU == 2) fac.g1 = fma(-fac.t, gp[NX], gp[NX + 1]);
                okl = okd;
              }
            }
          }
        }
        STAMP_SUB(12);
        if constexpr (kRow) {
          // the row chain (rowchain.h): the node lanes hand their stages to LDS records, every row runs
          // its instance's whole recursion, and node lane k takes step k's results back -- the same
          // operations as riccati_step below, so the same bits
          static_assert(!kDec && !kWsStash, "row chain: plain sequential recursion only");
          int rslot = (int)((threadIdx.x & 63) / (G * R)) * G * rowchain::kRec;
          asm volatile("" : "+v"(rslot));  // (not hoisted out of the solve loop: one register less there)
          double* rinst = rcbuf + rslot;
          // P_N = Sigma_x + delta, p_N = barrier gradient (node N's value function)
          auto terminal = [&](double* Pt, double* pt) __attribute__((always_inline)) {
            const double dl = (k == N) ? 1.0 : 0.0;
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
              for (int j = i; j < NX; ++j) Pt[symix(i, j, NX)] = (i == j) ? dl * (sgv[i] + delta) : 0.0;
              pt[i] = dl * gp[i];
            }
          };
          if (seq && (R == 1 || rho == 0)) {
            if (hasU) {
              rowchain::store_stage(rinst + k * rowchain::kRec, Hd, gp, Aop, Bop, cdef);
            } else if (hasX && k == N) {
              double PN[NP], pN[NX];
              terminal(PN, pN);
              rowchain::store_terminal(rinst + k * rowchain::kRec, PN, pN);
            }
          }
          // one wave per workgroup (G R <= 64): its LDS accesses complete in issue order, so the
          // hand-overs need only a compiler barrier, no s_barrier and no wait for the stores
          static_assert(G * R <= 64, "row chain: single-wave workgroups");
          asm volatile("" ::: "memory");
          STAMP_SUB(11);  // (diagnostic build: the chain itself as sub-phase 11, unused by this model)
          rowchain::run<G * R>(rinst, N);
          asm volatile("" ::: "memory");
          STAMP_SUB(12);
          // every node redoes its own step from node k+1's value function -- the chain's step k, the
          // same function on the same operands -- for its factors and P_k, all nodes at once.  P, p and
          // the factors are (re)set only here, so none of them is live across the chain (node N and
          // the lanes past it: P_N / zeros and no factors, as the sequential recursion leaves them),
          // and the stage Hessian is formed again from its parts (the delta barrier keeps the compiler
          // from holding the pre-chain copy across the chain instead)
          if (seq) {
            if (hasU) {
              double Pin_[NP], pin_[NX], Hk[NH];
              rowchain::load_next(rinst + (k + 1) * rowchain::kRec, Pin_, pin_);
              double dlt = delta;
              asm volatile("" : "+v"(dlt));
              const double* Hsrc = Model::hessW(ctx, Hs);
#pragma unroll
              for (int i = 0; i < NH; ++i) Hk[i] = Hsrc[i];
#pragma unroll
              for (int i = 0; i < NZ; ++i) Hk[symix(i, i, NZ)] += sgv[i] + dlt;
              (void)riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, false, AOneOf<Model>::value>(
                  Hk, gp, Aop, Bop, cdef, Pin_, pin_, P, p, fac);
            } else {
              terminal(P, p);
              fac = Fac<NX, NU>{};
            }
            okl = !hasU || fac_ok<NX, NU>(fac);
          }
        } else if constexpr (kRow6) {
          // the 6-state row chain (rowchain6.h): the node lanes write their stages (from the
          // workspace stash) into the LDS ring window by window, every row runs the instance's
          // recursion and stores each node's value function into that node's workspace slots, and
          // node lane k redoes its own step from node k+1's -- the chain's step k, the same
          // operations as riccati_step, so the same bits -- for its factors and P_k
          static_assert(!kDec && kWsStash, "6-state row chain: plain sequential recursion, workspace stash");
          auto fill = [&](int lo, int hi, bool top) __attribute__((always_inline)) {
            if (seq && hasU && k >= lo && k <= hi) {
              const double* r = wsrec();
              double Hs_[NH], sg_[NZ], A_[NX * NX], B_[NX * NU];
#pragma unroll
              for (int i = 0; i < NH; ++i) Hs_[i] = wsload(r, kRH + i);
#pragma unroll
              for (int i = 0; i < NZ; ++i) sg_[i] = wsload(r, kRS + i);
              ws_jac(A_, B_);
              rowchain6::store_node(tcache + (k - lo) * rowchain6::kRec, Hs_, sg_, delta, A_, B_, gp, cdef);
            }
            if (top && seq && hasX && k == N)
              rowchain6::store_terminal(tcache + (N - lo) * rowchain6::kRec, sgv, delta, gp);
          };
          double* out0 = a.ws + (long)kWsH * a.ws_stride + (gid - k) * kCS + kRP;  // node 0's slots
          STAMP_SUB(11);
          const bool early = rowchain6::run(tcache, out0, kCS, valid && seq, N, fill);
          __syncthreads();  // row 0's workspace stores, before the node lanes read them
          STAMP_SUB(12);
          if (early) {
            // a step's reduced Huu' failed the inertia test (the chain stopped there): the attempt
            // fails whatever the other steps give -- the same decision as fac_ok after the full chain
            okl = false;
          } else if (seq) {
            if (hasU) {
              double Pin_[NP], pin_[NX], Hj[NH], Aj[NX * NX], Bj[NX * NU];
              rowchain6::load_next(wsrec() + kCS + kRP, Pin_, pin_);
              ws_jac(Aj, Bj);
              const double* r = wsrec();
#pragma unroll
              for (int i = 0; i < NZ; ++i)
#pragma unroll
                for (int jj = i; jj < NZ; ++jj) {
                  const int t = symix(i, jj, NZ);
                  Hj[t] = wsload(r, kRH + t);
                  if (jj == i) Hj[t] += wsload(r, kRS + i) + delta;
                }
              (void)riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, false, AOneOf<Model>::value>(
                  Hj, gp, Aj, Bj, cdef, Pin_, pin_, P, p, fac);
            } else {
              const double dl = (k == N) ? 1.0 : 0.0;  // node N: P_N = Sigma_x + delta, p_N = gradient
#pragma unroll
              for (int i = 0; i < NX; ++i) {
#pragma unroll
                for (int j = i; j < NX; ++j) P[symix(i, j, NX)] = (i == j) ? dl * (sgv[i] + delta) : 0.0;
                p[i] = dl * gp[i];
              }
              fac = Fac<NX, NU>{};
            }
            okl = !hasU || fac_ok<NX, NU>(fac);
          }
        } else if constexpr (G <= 64) {
          if constexpr (kDec) {
            for (int j = N - 1; j >= jc; --j) {
              double pin_[NX];
#pragma unroll
              for (int i = 0; i < NX; ++i) pin_[i] = from_next(p[i]);
              if (seq && k == j) {
                dec_vector_step<NX, NU, Model::AMASK, Model::BMASK>(gp, Aop, Bop, vpc, pin_, p, fac);
                okl = okd;
              }
            }
          }
          // models with a long chain step (the workspace-stash models, one instance per wave): a
          // failed inertia test ends the chain early (below)
          constexpr bool kEarly = kWsStash && !kDec && G == 64;
          bool early = false;
          // the chain: one step per node, lane j only.  Models without the decoupled suffix take
          // the inertia verdict of their step from its factors after the chain, on all lanes at
          // once (fac_ok), so no lane-mask merge sits on the chain
#pragma unroll 2
          for (int j = min(N, jc) - 1; j >= 0; --j) {
            const bool cheap = reuse && j >= kb;
            double Pin_[NP], pin_[NX];
            if (!kDec || __any(!cheap)) {
#pragma unroll
              for (int i = 0; i < NP; ++i) Pin_[i] = from_next(P[i]);
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) pin_[i] = from_next(p[i]);
            if (seq && k == j) {
              if constexpr (kDec) {
                if (cheap) {  // group-uniform
                  dec_vector_step<NX, NU, Model::AMASK, Model::BMASK>(gp, Aop, Bop, vpc, pin_, p, fac);
                  okl = okd;
                } else {
                  okl = riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, kDec, AOneOf<Model>::value>(
                      Hd, gp, Aop, Bop, cdef, Pin_, pin_, P, p, fac);
                }
              } else if constexpr (kWsStash) {
                // this step's operands from the workspace (lane j only): no lane keeps its stage
                // Hessian and Jacobians in registers across the chain
                double Hj[NH], Aj[NX * NX], Bj[NX * NU];
                ws_jac(Aj, Bj);
                {
                  const double* r = wsrec();
#pragma unroll
                  for (int i = 0; i < NZ; ++i)
#pragma unroll
                    for (int jj = i; jj < NZ; ++jj) {
                      const int t = symix(i, jj, NZ);
                      Hj[t] = wsload(r, kRH + t);
                      if (jj == i) Hj[t] += wsload(r, kRS + i) + delta;
                    }
                }
                (void)riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, kDec, AOneOf<Model>::value>(
                    Hj, gp, Aj, Bj, cdef, Pin_, pin_, P, p, fac);
              } else {
                (void)riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, kDec, AOneOf<Model>::value>(
                    Hd, gp, Aop, Bop, cdef, Pin_, pin_, P, p, fac);
              }
            }
            // a step whose reduced Huu' is not positive definite decides the attempt: the KKT
            // matrix has the wrong inertia whatever the remaining steps give, so the chain stops
            // there (one instance per wave, so the verdict is the wave's).  Same decision, same
            // delta sequence as running the chain out (fac_ok is the test taken after the chain)
            if constexpr (kEarly) {
              if (__any(seq && k == j && !fac_ok<NX, NU>(fac))) {
                early = true;
                break;
              }
            }
          }
          if constexpr (!kDec)
            if (seq) okl = !early && (!hasU || fac_ok<NX, NU>(fac));
        } else {  // wave by wave, N-side first; the value function crosses waves through LDS
          const int wv = (int)(threadIdx.x >> 6);
          for (int ph = XWave<G>::W - 1; ph >= 0; --ph) {
            if (wv == ph) {
              const double* in = xw.prev();  // (P, p) of node 64 (ph + 1), written last phase
              const int jtop = 64 * ph + 63;
              if constexpr (kDec) {  // this wave's reused-suffix steps (see jc above)
                for (int j = min(N - 1, jtop); !sscan && j >= max(jc, 64 * ph); --j) {
                  double pin_[NX];
#pragma unroll
                  for (int i = 0; i < NX; ++i) pin_[i] = from_next(p[i]);
                  if (j == jtop && lane == 63)
#pragma unroll
                    for (int i = 0; i < NX; ++i) pin_[i] = in[NP + i];
                  if (seq && k == j) {
                    dec_vector_step<NX, NU, Model::AMASK, Model::BMASK>(gp, Aop, Bop, vpc, pin_, p, fac);
                    okl = okd;
                  }
                }
              }
              for (int j = min(min(N - 1, jtop), jc - 1); j >= 64 * ph; --j) {
                const bool cheap = reuse && j >= kb;
                double Pin_[NP], pin_[NX];
                if (!kDec || __any(!cheap)) {
#pragma unroll
                  for (int i = 0; i < NP; ++i) Pin_[i] = from_next(P[i]);
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) pin_[i] = from_next(p[i]);
                if (j == jtop && lane == 63) {
#pragma unroll
                  for (int i = 0; i < NP; ++i) Pin_[i] = in[i];
#pragma unroll
                  for (int i = 0; i < NX; ++i) pin_[i] = in[NP + i];
                }
                if (seq && k == j) {
                  if (cheap) {  // group-uniform
                    dec_vector_step<NX, NU, Model::AMASK, Model::BMASK>(gp, Aop, Bop, vpc, pin_, p, fac);
                    okl = okd;
                  }
                  else
                    okl = riccati_step<NX, NU, Model::AMASK, Model::BMASK, false, kDec, AOneOf<Model>::value>(Hd, gp, Aop, Bop, cdef, Pin_, pin_, P, p,
                                                                                         fac);
                }
              }
              if (ph > 0 && lane == 0) {
                double* out = xw.cur();
#pragma unroll
                for (int i = 0; i < NP; ++i) out[i] = P[i];
#pragma unroll
                for (int i = 0; i < NX; ++i) out[NP + i] = p[i];
              }
            }
            xw.sync();
          }
        }
      }
      STAMP_SUB(13);
      stash(true);
      // node 0: A_0 = 0 and no x blocks in stage 0 (interval 0 integrates from x0), so the step
      // gives P_0 = Sigma_x + delta and p_0 = the barrier gradient, as at node N; its factors
      // (Huu', gu', the inertia test) do not involve A_0 and stand as computed
      if (k == 0) {
#pragma unroll
        for (int i = 0; i < NX; ++i) {
#pragma unroll
          for (int j = i; j < NX; ++j) P[symix(i, j, NX)] = (i == j) ? sgv[i] + delta : 0.0;
          p[i] = gp[i];
        }
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) Pk[i] = P[i];
#pragma unroll
      for (int i = 0; i < NX; ++i) pk[i] = p[i];
      const bool ok = gall<G, G * R>(okl, xw);
      // Decoupled suffix of a multi-wave group (G > 64): the reused path sums the suffix's vector
      // part by the log-depth scan, the full recursion in chain order.  A fresh delta = 0
      // factorisation has just stored the suffix's P_k -- the bits the cross-launch cache would
      // hold -- so it is redone on the reused path (block-uniform; the scan's conditions): an
      // instance's result then does not depend on the cache state (a fresh handle, an earlier
      // launch's cache, a step of a multi-step launch, a device schedule that bypasses the cache)
      if constexpr (kDec && G > 64) {
        if (need && ok && !pcv && delta == 0.0 && kb < N && !a.lin.per_instance && a.tabseq == nullptr) {
          pcv = true;
          continue;
        }
      }
      // IPOPT inertia correction (Algorithm IC)
      if (need) {
        if (ok) {
          need = false;
          if (delta > 0.0) dw_last = delta;
          if (delta > 0.0) DIAG(0);
        } else {
          DIAG(1);
          if (first) delta = dw_last == 0.0 ? kDw0 : fmax(kDwMin, kKwMinus * dw_last);
          else delta *= dw_last == 0.0 ? kKwPlusBar : kKwPlus;
          first = false;
          if (delta > kDwMax) {
            need = false;
            failed = true;
          }
        }
      }
    }
    if (!done && failed) {
      done = true;
      status = 5;  // inertia correction failed (IPOPT Error_In_Step_Computation)
      its = it;
    }
    if constexpr (kDec) {
      pcv = !failed && delta == 0.0;  // Pk now holds a delta = 0 factorisation
      // publish it for later launches (every writer stores the same bits; readers accept only
      // the header of an earlier launch, so a half-written cache is never read)
      if (fresh_fac && pcv && pc_miss && pcache_ok(fs)) {
        if (k >= kb && k <= N)
#pragma unroll
          for (int i = 0; i < NP; ++i) a.pcache[(size_t)k * NP + i] = Pk[i];
        if (k == 0) {
          double* hdr = a.pcache + (size_t)(N + 1) * NP;
          hdr[0] = a.pc_epoch;
          hdr[1] = a.pc_gen;
          hdr[2] = (double)kb;
        }
      }
    }
    riccati_gains<NX, NU>(fac, Kk, kfk);  // all lanes at once
    if (k == 0)  // Hux'_0 = 0 (A_0 = 0): no feedback on X_0
#pragma unroll
      for (int i = 0; i < NU * NX; ++i) Kk[i] = 0.0;

    STAMP(4);
    phase();
    // ------------------------------------------------------------ forward sweep: dw (lane k-1 -> k)
    // (a lambda: the second-order correction re-runs it with other right-hand sides)
    auto forward = [&](const double* cc_, const double* kf_, const double* pv_, const double* c0v_, double* dzo_,
                       double* dlo_) __attribute__((always_inline)) {
      // closed-loop map of the step, node-parallel (off the sequential chain):
      // dx_{k+1} = (A + B K) dx_k + (c + B k_f);  du_k = k_f + K dx_k afterwards
      double Acl[NX * NX], ccl[NX];
      double Aw_[kWsStash ? NX * NX : 1], Bw_[kWsStash ? NX * NU : 1];
      const double* Af_ = Model::jacA(ctx, A);
      const double* Bf_ = Model::jacB(ctx, Bm);
      if constexpr (kWsStash) {
        ws_jac(Aw_, Bw_);
        Af_ = Aw_;
        Bf_ = Bw_;
      }
#pragma unroll
      for (int r = 0; r < NX; ++r) {
        double acc = cc_[r];
#pragma unroll
        for (int l = 0; l < NU; ++l)
          if (Model::BMASK & (1ull << (r * NU + l))) acc = fma(Bf_[r * NU + l], kf_[l], acc);
        ccl[r] = acc;
#pragma unroll
        for (int m = 0; m < NX; ++m) {
          double e = (Model::AMASK & (1ull << (r * NX + m))) ? Af_[r * NX + m] : 0.0;
#pragma unroll
          for (int l = 0; l < NU; ++l)
            if (Model::BMASK & (1ull << (r * NU + l))) e = fma(Bf_[r * NU + l], Kk[l * NX + m], e);
          Acl[r * NX + m] = e;
        }
      }
      {
        // dx_k = T_{k-1}( ... T_0(c0)) with affine T_j(x) = Acl_j x + ccl_j: an inclusive
        // parallel prefix of map compositions (log2 GW levels per wave, all lanes busy) instead
        // of N+1 dependent steps.  Lane k starts with T_{k-1} (lane 0: the constant map c0) and
        // composes with the partial map of its DPP partner at each level: Kogge-Stone inside
        // each 16-lane row, then the previous rows' totals by row broadcasts (scan_partner; the
        // ds_bpermute version of the same scan, Hillis-Steele over lane k-d: config 2 16.3 us per
        // IPM iteration against 15.8 us with the DPP partners, config 3 35.0 against 33.7 us).
        // Multi-wave groups scan every wave at once; the first lane of wave w gets
        // T_{64w-1} from wave w-1 through LDS, and the waves' partial results are chained
        // by one LDS handoff of dx per wave boundary.
        constexpr int NM = NX * NX + NX;
        constexpr int GW = G < 64 ? G : 64;  // lanes scanned per wave
        const int wv = G > 64 ? (int)(threadIdx.x >> 6) : 0;
        double Am[NX * NX], cm[NX];
        {
          double own[NM], prv[NM];
#pragma unroll
          for (int i = 0; i < NX * NX; ++i) own[i] = Acl[i];
#pragma unroll
          for (int i = 0; i < NX; ++i) own[NX * NX + i] = ccl[i];
#pragma unroll
          for (int i = 0; i < NM; ++i) prv[i] = from_prev(own[i]);
          if constexpr (G > 64) {  // lane 0 of wave w > 0: T_{64w-1} lives on lane 63 of wave w-1
            double* b = xw.cur();
            if (lane == 63 && wv < XWave<G>::W - 1)
#pragma unroll
              for (int i = 0; i < NM; ++i) b[wv * kXchStride + i] = own[i];
            xw.sync();
            if (lane == 0 && wv > 0)
#pragma unroll
              for (int i = 0; i < NM; ++i) prv[i] = xw.prev()[(wv - 1) * kXchStride + i];
          }
          // lane 1 takes only T_0's constant part: dx_1 = B_0 du_0 + c_1 does not depend on dx_0
          // (interval 0 integrates from x0, A_0 = 0)
#pragma unroll
          for (int i = 0; i < NX * NX; ++i) Am[i] = (k <= 1) ? 0.0 : prv[i];
#pragma unroll
          for (int i = 0; i < NX; ++i) cm[i] = (k == 0) ? c0v_[i] : prv[NX * NX + i];
        }
        const int kw = k & (GW - 1);  // position inside the wave
        // one level: compose with the partial map of the DPP partner (collectives.h scan_partner)
        auto level = [&](auto dc) __attribute__((always_inline)) {
          constexpr int d = decltype(dc)::value;
          if constexpr (d < GW) {
          double Ao[NX * NX], co[NX];
#pragma unroll
          for (int i = 0; i < NX * NX; ++i) Ao[i] = scan_partner<d>(Am[i]);
#pragma unroll
          for (int i = 0; i < NX; ++i) co[i] = scan_partner<d>(cm[i]);
          if (scan_takes<d>(kw)) {  // compose: (Am, cm) o (Ao, co)
            double An[NX * NX], cn[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
              double acc = cm[r];
#pragma unroll
              for (int m = 0; m < NX; ++m) acc = fma(Am[r * NX + m], co[m], acc);
              cn[r] = acc;
#pragma unroll
              for (int c = 0; c < NX; ++c) {
                double e = Am[r * NX] * Ao[c];
#pragma unroll
                for (int m = 1; m < NX; ++m) e = fma(Am[r * NX + m], Ao[m * NX + c], e);
                An[r * NX + c] = e;
              }
            }
#pragma unroll
            for (int i = 0; i < NX * NX; ++i) Am[i] = An[i];
#pragma unroll
            for (int i = 0; i < NX; ++i) cm[i] = cn[i];
          }
          }
        };
        level(std::integral_constant<int, 1>{});
        level(std::integral_constant<int, 2>{});
        level(std::integral_constant<int, 4>{});
        level(std::integral_constant<int, 8>{});
        level(std::integral_constant<int, 16>{});
        level(std::integral_constant<int, 32>{});
        if constexpr (G > 64) {
          // wave w's lanes hold maps dx_{64w-1} -> dx_k; chain the waves in order
          for (int ph = 1; ph < XWave<G>::W; ++ph) {
            double* b = xw.cur();
            if (wv == ph - 1 && lane == 63)
#pragma unroll
              for (int i = 0; i < NX; ++i) b[i] = cm[i];
            xw.sync();
            if (wv == ph) {
              const double* in = xw.prev();
              double cn[NX];
#pragma unroll
              for (int r = 0; r < NX; ++r) {
                double acc = cm[r];
#pragma unroll
                for (int m = 0; m < NX; ++m) acc = fma(Am[r * NX + m], in[m], acc);
                cn[r] = acc;
              }
#pragma unroll
              for (int i = 0; i < NX; ++i) cm[i] = cn[i];
            }
          }
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) dzo_[i] = cm[i];
      }
      // du_k = k_f + K dx_k on all lanes at once (the last node has no control)
#pragma unroll
      for (int l = 0; l < NU; ++l) {
        double acc = kf_[l];
#pragma unroll
        for (int m = 0; m < NX; ++m) acc = fma(Kk[l * NX + m], dzo_[m], acc);
        dzo_[NX + l] = (k < N) ? acc : 0.0;
      }
      // lambda+ = P_k dx_k + p_k (node-parallel, after the sequential sweep)
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        double acc = pv_[i];
#pragma unroll
        for (int m = 0; m < NX; ++m) acc = fma(Pk[symix(i, m, NX)], dzo_[m], acc);
        dlo_[i] = acc - lam[i];
      }
      if (!hasX) {
#pragma unroll
        for (int i = 0; i < NZ; ++i) dzo_[i] = 0.0;
#pragma unroll
        for (int i = 0; i < NX; ++i) dlo_[i] = 0.0;
      }
    };
    forward(cdef, kfk, pk, c0, dz, dlam);

    STAMP(5);
    phase();
    // ------------------------------------------------------------ bound-dual step, fraction to boundary
    double amax_l = 1.0, az_l = 1.0, tiny_l = -1.0, gd_l = 0.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      dzL[i] = dzU[i] = 0.0;
      const double rdz = rcp64(dz[i]);
      if (hL[i]) {
        const double s = z[i] - lb[i], rs = rcp64(s);
        dzL[i] = fma(mu, rs, -zL[i]) - zL[i] * rs * dz[i];
        if (dz[i] < 0) amax_l = fmin(amax_l, -tau * s * rdz);
        if (dzL[i] < 0) az_l = fmin(az_l, -tau * zL[i] * rcp64(dzL[i]));
      }
      if (hU[i]) {
        const double s = ub[i] - z[i], rs = rcp64(s);
        dzU[i] = fma(mu, rs, -zU[i]) + zU[i] * rs * dz[i];
        if (dz[i] > 0) amax_l = fmin(amax_l, tau * s * rdz);
        if (dzU[i] < 0) az_l = fmin(az_l, -tau * zU[i] * rcp64(dzU[i]));
      }
      const bool own = (i < NX) ? hasX : hasU;
      // IPOPT's tiny step test max |dz_i| / (1 + |z_i|) < 10 eps as the sign of
      // |dz_i| - 10 eps (1 + |z_i|) (one fma, no reciprocal)
      tiny_l = qmax(tiny_l, own ? fma(-10.0 * kEps, 1.0 + fabs(z[i]), fabs(dz[i])) : -1.0);
      if (own) gd_l += gp[i] * dz[i];
    }
    // amax, az (min), gd (sum) and the tiny-step test (max over the group < 0) in one exchange
    double fr[4] = {amax_l, az_l, gd_l, tiny_l < 0.0 ? 1.0 : 0.0};
    if constexpr (G > 64) {
      greduce_n<G, 2, 2, 0, 3>(fr, xw);
    } else {
      greduce_n<G, 2, 2, 0>(fr, xw);
      fr[3] = gall<G, G * R>(tiny_l < 0.0, xw) ? 1.0 : 0.0;
    }
    const double amax = fr[0];
    double az = fr[1];  // dual step length (a second-order correction replaces it)
    const bool tinystep = fr[3] > 0.5;
    if (!done && amax < 1.0) DIAG(4);
    if (!done && tinystep) DIAG(5);
    const double gd = fr[2];

    STAMP(6);
    phase();
    // ------------------------------------------------------------ filter line search
    double thk_l = 0, phk_l = (hasU ? fs * qv : 0.0) - mu * (lz_ok ? Lz : barrier_logsum<NZ>(z, lb, ub, hL, hU));
    lz_ok = false;
#pragma unroll
    for (int i = 0; i < NX; ++i) thk_l += fabs(cdef[i]) + fabs(c0[i]);
    double tp[2] = {thk_l, phk_l};
    greduce_n<G, 0, 0>(tp, xw);
    const double thk = tp[0], phk = tp[1];
    double alpha = amax;
    bool searching = !done && !tinystep && !(kRes && soft);
    bool accepted = !done && tinystep;
    bool ftype = tinystep;
    tiny_flag = !done && tinystep;
    bool trial_fresh = false;  // accepted at the first trial, which evaluated derivatives
    bool lastrej_f = false;    // the last rejected trial passed the sufficient decrease test but not the filter
    bool soft_pd = false;      // (kSoftInline) accepted by the primal-dual error reduction (filter kept)
    soft_tried = false;
    // switching condition alpha (-gd)^s_phi > delta theta^s_theta  <=>  alpha > sw_a with
    // sw_a = delta theta^s_theta / (-gd)^s_phi -- also the third term of alpha_min; one exp of
    // logs, loop-invariant over the trials.  A long dependent chain of scalar operations: the
    // models whose first trial evaluates derivatives form it beside that evaluation (same basic
    // block, so the scheduler interleaves the two), the others here
    double sw_a = 0.0, amin = kGammaAlpha * kGammaTheta;
    bool sw_set = false;
    auto switching = [&]() __attribute__((always_inline)) {
      if (gd < 0) {
        static_assert(kDeltaSw == 1.0, "log(delta) = 0");
        sw_a = exp_fd(kSTheta * log_fd(thk) - kSPhi * log_fd(-gd));
        amin = kGammaAlpha * fmin(kGammaTheta, fmin(kGammaPhi * thk / (-gd), sw_a));
      }
      sw_set = true;
    };
    constexpr bool kSwInSearch = Model::kEvalInSearch && !Model::kSOC;
    if constexpr (!kSwInSearch) switching();
    double Lt0 = 0.0;        // (kEvalInSearch) this lane's barrier log-sum at the first trial point
    bool acc0 = false;       // accepted at the first trial of the filter line search
    if constexpr (!Model::kSOC) {
    // one trial point: the barrier term, the group sums of theta and phi, the filter test and
    // IPOPT's acceptance (sufficient decrease -- switching condition + Armijo, or theta/phi
    // decrease -- then the filter: IPOPT's order, which decides whether a rejection was the filter's)
    auto trial_accept = [&](int ls, double tht_l, double pht_l, const double* zt) __attribute__((always_inline)) {
      const double Lt = barrier_logsum<NZ>(zt, lb, ub, hL, hU);
      if (ls == 0) Lt0 = Lt;
      pht_l -= mu * Lt;
      double tp_[2] = {tht_l, pht_l};
      greduce_n<G, 0, 0>(tp_, xw);
      const double tht = tp_[0], pht = tp_[1];
      const bool infilter = filt.contains(tht, pht, xw);
      if (searching) {
        bool acc = isfinite(pht) && isfinite(tht) && tht <= theta_max;
        bool ft = false;
        if (acc) {
          const bool sw = gd < 0 && alpha > sw_a;
          if (thk <= theta_min && sw) {
            acc = pht - phk <= kEtaPhi * alpha * gd + 10.0 * kEps * fabs(phk);
            ft = acc;
          } else {
            acc = tht <= (1.0 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10.0 * kEps * fabs(phk);
          }
        }
        if (acc && infilter) {
          acc = false;
          lastrej_f = true;
        } else if (!acc) {
          lastrej_f = false;
        }
        if (infilter) DIAG(6);
        if (acc) {
          searching = false;
          accepted = true;
          ftype = ft;
          trial_fresh = Model::kEvalInSearch && ls == 0;
          acc0 = ls == 0;
          if (ft) DIAG(7);
        } else {
          DIAG(2);
          alpha *= 0.5;
          if (alpha < amin) searching = false;  // would need restoration
        }
      }
    };
    // a trial's constraint violation and objective by the value function (every lane: group_next)
    auto trial_value_sums = [&](const double* zt, double& tht_l, double& pht_l) __attribute__((always_inline)) {
      double xtn[NX];
      group_next<G, NX>(zt, xtn, xw);
      double xft[NX], qt, ze[NZ];
      stage_point(zt, ze);
      Model::value(ma, ctx, ze, xft, qt);
      if (hasU) {
#pragma unroll
        for (int i = 0; i < NX; ++i) tht_l += fabs(xft[i] - xtn[i]);
        pht_l = fs * qt;
      }
      if (valid && k == 0)
#pragma unroll
        for (int i = 0; i < NX; ++i) tht_l += fabs(x0[i] - zt[i]);
    };
    // the first trial (alpha = alpha_max) as straight-line code ahead of the backtracking loop:
    // the usual iteration accepts it and runs no loop control
    if (__any(searching)) {
      phase();
      double zt[NZ];
#pragma unroll
      for (int i = 0; i < NZ; ++i) zt[i] = fma(alpha, dz[i], z[i]);  // the update's exact expression
      double tht_l = 0, pht_l = 0;
      if constexpr (Model::kEvalInSearch) {
        if (searching) {  // group-uniform (block-uniform for multi-wave groups)
          double lt[NX];
#pragma unroll
          for (int i = 0; i < NX; ++i) lt[i] = fma(alpha, dlam[i], lam[i]);
#ifdef MPCX_STAMP_EVAL
          STAMP(9);  // diagnostic: the trial's evaluation accumulates into phase 9
#endif
          eval_at(zt, lt);
          if constexpr (kSwInSearch) switching();
#ifdef MPCX_STAMP_EVAL
          STAMP(6);
#endif
          fresh = false;  // until accepted
#pragma unroll
          for (int i = 0; i < NX; ++i) tht_l += fabs(cdef[i]) + fabs(c0[i]);
          pht_l = fs * qv;  // masked to 0 without an interval
        }
      } else {
        trial_value_sums(zt, tht_l, pht_l);
      }
      trial_accept(0, tht_l, pht_l, zt);
    }
    // backtracking: the further trials evaluate values only
    for (int ls = 1; ls < 80; ++ls) {
      if (!__any(searching)) break;
      phase();
      double zt[NZ];
#pragma unroll
      for (int i = 0; i < NZ; ++i) zt[i] = fma(alpha, dz[i], z[i]);
      double tht_l = 0, pht_l = 0;
      trial_value_sums(zt, tht_l, pht_l);
      trial_accept(ls, tht_l, pht_l, zt);
    }
    if constexpr (kSoftInline) {
      // ---- IPOPT's soft restoration step (resto.h step 1), taken here, out of the hot path,
      //      once the filter line search has failed or instead of it in the soft restoration
      //      phase: primal and dual variables take the same step min(alpha_max, alpha_z),
      //      accepted by the original criteria (the soft phase then ends) or by a reduction of
      //      the barrier problem's primal-dual error by kSoftResto (the filter is left as it is);
      //      at most kMaxSoftResto of them in a row.  Both primal-dual errors need derivatives,
      //      at the current point (the failed search's first trial replaced them) and at the
      //      trial point: ONE evaluation site run twice (no second copy of the model code).
      const bool want = res_on && !done && !tinystep && !accepted;  // group-uniform
      if (MPCX_COLD(__any(want))) {
        bool go = false;
        if (want) {
          if (soft) {
            go = ++soft_count <= kMaxSoftResto;
          } else {
            soft = true;
            soft_count = 0;
            go = true;
          }
          soft_tried = !go;
          DIAG(12);
        }
        if (__any(go)) {
          if (!sw_set) switching();  // (a soft phase skips the filter search)
          const double as = fmin(amax, az);
          double zt[NZ], lt[NX];
#pragma unroll
          for (int i = 0; i < NZ; ++i) zt[i] = fma(as, dz[i], z[i]);
#pragma unroll
          for (int i = 0; i < NX; ++i) lt[i] = fma(as, dlam[i], lam[i]);
          double pd[2] = {0.0, 0.0}, tht = 0.0, pht = 0.0;
#pragma unroll 1
          for (int e = 0; e < 2; ++e) {  // e = 0: current point, e = 1: trial point
            double ze[NZ], le[NX], zLe[NZ], zUe[NZ];
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
              ze[i] = e ? zt[i] : z[i];
              zLe[i] = e ? fma(as, dzL[i], zL[i]) : zL[i];
              zUe[i] = e ? fma(as, dzU[i], zU[i]) : zU[i];
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) le[i] = e ? lt[i] : lam[i];
            eval_at(ze, le);
            // primal-dual error of the barrier problem (resto.h pd_error: 1-norms, its order)
            double lnx[NX], r[NZ];
            group_next<G, NX>(le, lnx, xw);
#pragma unroll
            for (int i = 0; i < NZ; ++i) r[i] = 0;
            if (hasX) {
#pragma unroll
              for (int i = 0; i < NX; ++i) r[i] = gq[i] - le[i];
              if (hasU) {
                if (k > 0)  // (X_0 enters only g_0)
#pragma unroll
                  for (int j = 0; j < NX; ++j)
#pragma unroll
                    for (int m = 0; m < NX; ++m)
                      if (Model::AMASK & (1ull << (m * NX + j)))
                        r[j] = fma(Model::jacA(ctx, A)[m * NX + j], lnx[m], r[j]);
#pragma unroll
                for (int l = 0; l < NU; ++l) {
                  double acc = gq[NX + l];
#pragma unroll
                  for (int m = 0; m < NX; ++m)
                    if (Model::BMASK & (1ull << (m * NU + l))) acc = fma(Model::jacB(ctx, Bm)[m * NU + l], lnx[m], acc);
                  r[NX + l] = acc;
                }
              }
            }
            double pdl = 0.0, thl = 0.0;
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
              pdl += fabs(r[i] + (zUe[i] - zLe[i]));
              if (hL[i]) pdl += fabs((ze[i] - lb[i]) * zLe[i] - mu);
              if (hU[i]) pdl += fabs((ub[i] - ze[i]) * zUe[i] - mu);
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
              pdl += fabs(cdef[i]) + fabs(c0[i]);
              thl += fabs(cdef[i]) + fabs(c0[i]);
            }
            pd[e] = gsum<G>(pdl, xw);
            if (e == 1) {
              tht = gsum<G>(thl, xw);
              pht = gsum<G>(fs * qv - mu * barrier_logsum<NZ>(zt, lb, ub, hL, hU), xw);
            }
          }
          fresh = false;  // the arrays hold the trial point's evaluation (kept if it is accepted)
          const bool infilter = filt.contains(tht, pht, xw);
          if (go) {
            // the original criteria first ...
            bool acc = isfinite(pht) && isfinite(tht) && tht <= theta_max;
            bool ft = false;
            if (acc) {
              if (thk <= theta_min && gd < 0 && as > sw_a) {
                acc = pht - phk <= kEtaPhi * as * gd + 10.0 * kEps * fabs(phk);
                ft = acc;
              } else {
                acc = tht <= (1.0 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10.0 * kEps * fabs(phk);
              }
            }
            if (acc && !infilter) {  // a regular step: the soft phase ends
              accepted = true;
              ftype = ft;
              lastrej_f = false;
              soft = false;
              soft_count = 0;
            } else if (pd[1] <= kSoftResto * pd[0]) {  // ... then the primal-dual error reduction
              accepted = true;
              soft_pd = true;
            } else {
              soft_tried = true;
            }
            if (accepted) {
              alpha = az = as;  // primal and dual variables take the same step
              trial_fresh = true;
              acc0 = false;
            }
          }
        }
      }
    }
    } else {  // models with the second-order correction (their trials evaluate values only)
    // trial point zt: constraint violation, barrier objective, filter membership (group sums);
    // ct / ct0 receive the trial's own constraint values (interval k, and g_0 on lane 0)
    auto trial_value = [&](const double* zt, double& tht, double& pht, bool& infilter, double* ct, double* ct0)
                           __attribute__((always_inline)) {
      double xtn[NX];
      group_next<G, NX>(zt, xtn, xw);
      double xft[NX], qt, ze[NZ];
      stage_point(zt, ze);
      Model::value(ma, ctx, ze, xft, qt);
      double tht_l = 0, pht_l = 0;
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        ct[i] = hasU ? xft[i] - xtn[i] : 0.0;
        ct0[i] = (valid && k == 0) ? x0[i] - zt[i] : 0.0;
      }
      if (hasU) {
#pragma unroll
        for (int i = 0; i < NX; ++i) tht_l += fabs(ct[i]);
        pht_l = fs * qt;
      }
      if (valid && k == 0)
#pragma unroll
        for (int i = 0; i < NX; ++i) tht_l += fabs(ct0[i]);
      pht_l -= mu * barrier_logsum<NZ>(zt, lb, ub, hL, hU);
      double tp_[2] = {tht_l, pht_l};
      greduce_n<G, 0, 0>(tp_, xw);
      tht = tp_[0];
      pht = tp_[1];
      infilter = filt.contains(tht, pht, xw);
    };
    // acceptance of a trial point for step length al (W&B 2006 A-5.4): sufficient decrease
    // (switching condition + Armijo, or theta/phi decrease), then the filter -- IPOPT's order,
    // which decides whether a rejection was the filter's
    auto acceptable = [&](double tht, double pht, bool infilter, double al, bool& ft) __attribute__((always_inline)) {
      bool acc = isfinite(pht) && isfinite(tht) && tht <= theta_max;
      ft = false;
      if (acc) {
        const bool sw = gd < 0 && al > sw_a;
        if (thk <= theta_min && sw) {
          acc = pht - phk <= kEtaPhi * al * gd + 10.0 * kEps * fabs(phk);
          ft = acc;
        } else {
          acc = tht <= (1.0 - kGammaTheta) * thk || pht <= phk - kGammaPhi * thk + 10.0 * kEps * fabs(phk);
        }
      }
      if (acc && infilter) {
        acc = false;
        lastrej_f = true;
      } else if (!acc) {
        lastrej_f = false;
      }
      return acc;
    };
    for (int ls = 0; ls < 80; ++ls) {
      if (!__any(searching)) break;
      phase();
      double zt[NZ];
#pragma unroll
      for (int i = 0; i < NZ; ++i) zt[i] = fma(alpha, dz[i], z[i]);  // the update's exact expression
      double tht, pht;
      bool infilter;
      double ct[NX], ct0[NX];  // constraint values at the trial point (value path)
      trial_value(zt, tht, pht, infilter, ct, ct0);
      bool soc_want = false;  // first trial rejected with more infeasibility: second-order correction
      if (searching) {
        bool ft;
        const bool acc = acceptable(tht, pht, infilter, alpha, ft);
        if (infilter) DIAG(6);
        if (acc) {
          searching = false;
          accepted = true;
          ftype = ft;
          if (ft) DIAG(7);
        } else {
          DIAG(2);
          DIAG_IF(ls == 0 && tht >= thk, 10);
          soc_want = ls == 0 && tht >= thk;
          if (!soc_want) {
            alpha *= 0.5;
            if (alpha < amin) searching = false;  // would need restoration
          }
        }
      }
      {
        // IPOPT's second-order correction (W&B 2006 A-5.7-A-5.9, max_soc = 4, kappa_soc = 0.99):
        // re-solve the Newton system (same factorisation) with the constraint residual
        // c_soc = alpha c(x_k) + c(x_trial), step to the boundary along the correction, and
        // test it with the first trial's step length; accumulate and retry while the
        // infeasibility keeps shrinking by kappa_soc
        if (ls == 0 && __any(soc_want)) {
          bool son = soc_want;
          double cs[NX], cs0[NX];
#pragma unroll
          for (int i = 0; i < NX; ++i) {
            cs[i] = fma(alpha, cdef[i], ct[i]);
            cs0[i] = fma(alpha, c0[i], ct0[i]);
          }
          double th_old = thk;
          double Pn1[NP];  // P_{k+1}
          group_next<G, NP>(Pk, Pn1, xw);
          for (int ps = 0; ps < 4; ++ps) {
            if (!__any(son)) break;
            // backward recursion of the value function's linear part only (the factorisation
            // P_k, K_k, Huu' is the current iteration's): p_k = gx + K^T gu with
            // s = p_{k+1} + P_{k+1} c_soc, gx = gp_x + A^T s, gu = gp_u + B^T s; k_f = -Huu'^-1 gu
            double pv[NX], kfs[NU];
#pragma unroll
            for (int i = 0; i < NX; ++i) pv[i] = (k == N) ? gp[i] : 0.0;
#pragma unroll
            for (int l = 0; l < NU; ++l) kfs[l] = 0.0;
            auto soc_step = [&](const double* pin) __attribute__((always_inline)) {
              const double* Aop = Model::jacA(ctx, A);
              const double* Bop = Model::jacB(ctx, Bm);
              double Aw_[kWsStash ? NX * NX : 1], Bw_[kWsStash ? NX * NU : 1];
              if constexpr (kWsStash) {
                ws_jac(Aw_, Bw_);
                Aop = Aw_;
                Bop = Bw_;
              }
              double sv[NX], gu[NU];
#pragma unroll
              for (int i = 0; i < NX; ++i) {
                double acc = pin[i];
#pragma unroll
                for (int m = 0; m < NX; ++m) acc = fma(Pn1[symix(i, m, NX)], cs[m], acc);
                sv[i] = acc;
              }
#pragma unroll
              for (int l = 0; l < NU; ++l) {
                double acc = gp[NX + l];
#pragma unroll
                for (int m = 0; m < NX; ++m)
                  if (Model::BMASK & (1ull << (m * NU + l))) acc = fma(Bop[m * NU + l], sv[m], acc);
                gu[l] = acc;
              }
#pragma unroll
              for (int i = 0; i < NX; ++i) {
                double acc = gp[i];
#pragma unroll
                for (int m = 0; m < NX; ++m)
                  if (Model::AMASK & (1ull << (m * NX + i))) acc = fma(Aop[m * NX + i], sv[m], acc);
#pragma unroll
                for (int l = 0; l < NU; ++l) acc = fma(Kk[l * NX + i], gu[l], acc);
                pv[i] = acc;
              }
              if constexpr (NU == 1) {
                kfs[0] = -fac.r0 * gu[0];
              } else {
                const double z1 = fac.r1 * fma(-fac.t, gu[0], gu[1]);
                kfs[1] = -z1;
                kfs[0] = -fma(fac.r0, gu[0], -fac.t * z1);
              }
            };
            if constexpr (G <= 64) {
              for (int j = N - 1; j >= 0; --j) {
                double pin[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) pin[i] = from_next(pv[i]);
                if (k == j) soc_step(pin);
              }
            } else {  // wave by wave, N-side first; p crosses waves through LDS
              const int wv = (int)(threadIdx.x >> 6);
              for (int ph = XWave<G>::W - 1; ph >= 0; --ph) {
                if (wv == ph) {
                  const double* in = xw.prev();
                  const int jtop = 64 * ph + 63;
                  for (int j = min(N - 1, jtop); j >= 64 * ph; --j) {
                    double pin[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) pin[i] = from_next(pv[i]);
                    if (j == jtop && lane == 63)
#pragma unroll
                      for (int i = 0; i < NX; ++i) pin[i] = in[i];
                    if (k == j) soc_step(pin);
                  }
                  if (ph > 0 && lane == 0) {
                    double* out = xw.cur();
#pragma unroll
                    for (int i = 0; i < NX; ++i) out[i] = pv[i];
                  }
                }
                xw.sync();
              }
            }
            if (k == 0)  // p_0 of the correction: the barrier gradient (A_0 = 0, K_0 = 0)
#pragma unroll
              for (int i = 0; i < NX; ++i) pv[i] = gp[i];
            double dzs[NZ], dls[NX];
            forward(cs, kfs, pv, cs0, dzs, dls);
            // primal and dual fraction to the boundary along the correction
            double am_l = 1.0, azs_l = 1.0, dzLs[NZ], dzUs[NZ];
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
              dzLs[i] = dzUs[i] = 0.0;
              const double rdz = rcp64(dzs[i]);
              if (hL[i]) {
                const double sl = z[i] - lb[i], rs = rcp64(sl);
                dzLs[i] = fma(mu, rs, -zL[i]) - zL[i] * rs * dzs[i];
                if (dzs[i] < 0) am_l = fmin(am_l, -tau * sl * rdz);
                if (dzLs[i] < 0) azs_l = fmin(azs_l, -tau * zL[i] * rcp64(dzLs[i]));
              }
              if (hU[i]) {
                const double su = ub[i] - z[i], rs = rcp64(su);
                dzUs[i] = fma(mu, rs, -zU[i]) + zU[i] * rs * dzs[i];
                if (dzs[i] > 0) am_l = fmin(am_l, tau * su * rdz);
                if (dzUs[i] < 0) azs_l = fmin(azs_l, -tau * zU[i] * rcp64(dzUs[i]));
              }
            }
            const double as = gmin<G>(am_l, xw), azs = gmin<G>(azs_l, xw);
            double zs[NZ];
#pragma unroll
            for (int i = 0; i < NZ; ++i) zs[i] = fma(as, dzs[i], z[i]);
            double ths, phs, cts[NX], cts0[NX];
            bool infs;
            trial_value(zs, ths, phs, infs, cts, cts0);
#ifdef MPCX_DEBUG_PRINT
            if (inst == 0 && k == 0)
              printf("SOC it=%d ps=%d son=%d alpha0=%g as=%g thk=%.17g phk=%.17g ths=%.17g phs=%.17g infs=%d fnext=%d\n", it,
                     ps, (int)son, alpha, as, thk, phk, ths, phs, (int)infs, filt.next);
#endif
            if (son) {
              bool ft;
              if (acceptable(ths, phs, infs, alpha, ft)) {  // tested with the first trial's alpha
                son = false;
                searching = false;
                accepted = true;
                ftype = ft;
                alpha = as;
                az = azs;
#pragma unroll
                for (int i = 0; i < NZ; ++i) {
                  dz[i] = dzs[i];
                  dzL[i] = dzLs[i];
                  dzU[i] = dzUs[i];
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) dlam[i] = dls[i];
                DIAG(11);
              } else if (ps == 3 || ths > 0.99 * th_old) {
                son = false;
              } else {
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                  cs[i] = fma(as, cs[i], cts[i]);
                  cs0[i] = fma(as, cs0[i], cts0[i]);
                }
                th_old = ths;
              }
            }
          }
          if (soc_want && searching) {  // correction failed: backtrack along the original direction
            alpha *= 0.5;
            if (alpha < amin) searching = false;
          }
        }
      }
    }
    }
    // ---- soft restoration / restoration phase (resto.h): the failed line search's iterate, its
    //      Newton step and the loop's scalars go to the workspace; the solve launch parks the
    //      instance there (the resume launch recovers and continues it), the resume launch
    //      recovers at the top of its next pass
    bool handled = false;
    if constexpr (kRes) {
      // (kSoftInline: the soft restoration step ran in the line search above; what is left is the
      // restoration phase proper, which IPOPT enters unless the point is acceptable)
      const bool need_rec = kSoftInline ? (res_on && !done && !tinystep && !accepted && !acceptable_now)
                                        : (res_on && !done && !tinystep && (soft || !accepted));
      if (MPCX_COLD(__any(need_rec))) {
        if (need_rec) {
          DIAG(12);
          // the workspace addresses are made opaque here, so that the compiler cannot hoist their
          // computation out of the solve loop (45 loop-invariant 64-bit addresses held in
          // registers through every iteration: +146 VGPR spills on the unicycle kernel)
          double* wsl = a.ws + gid;
          long wst = a.ws_stride;
          asm volatile("" : "+v"(wsl), "+v"(wst));
          auto W = [&](int i) __attribute__((always_inline)) -> double& { return wsl[(long)i * wst]; };
#pragma unroll
          for (int i = 0; i < NZ; ++i) {
            W(RestoWs::XZ + i) = z[i];
            W(RestoWs::XZL(NX, NZ) + i) = zL[i];
            W(RestoWs::XZU(NX, NZ) + i) = zU[i];
            W(RestoWs::XDZ(NX, NZ) + i) = dz[i];
            W(RestoWs::XDZL(NX, NZ) + i) = dzL[i];
            W(RestoWs::XDZU(NX, NZ) + i) = dzU[i];
          }
#pragma unroll
          for (int i = 0; i < NX; ++i) {
            W(RestoWs::XL(NZ) + i) = lam[i];
            W(RestoWs::XDL(NX, NZ) + i) = dlam[i];
            W(RestoWs::XX0(NX, NZ) + i) = x0[i];
          }
          constexpr int S = RestoWs::SC(NX, NZ);
          W(S + RestoWs::sFS) = fs;
          W(S + RestoWs::sMU) = mu;
          W(S + RestoWs::sTAU) = tau;
          W(S + RestoWs::sTHMAX) = theta_max;
          W(S + RestoWs::sTHMIN) = theta_min;
          W(S + RestoWs::sDWLAST) = dw_last;
#pragma unroll
          for (int j = 0; j < FilterLds<G>::S; ++j) {
            W(S + RestoWs::sFTH + j) = filt.th(j);
            W(S + RestoWs::sFPH + j) = filt.ph(j);
          }
          W(S + RestoWs::sFNEXT) = filt.next;
          W(S + RestoWs::sFN) = filt.n;
          W(S + RestoWs::sFREJ) = frej;
          W(S + RestoWs::sNFRESET) = nfreset;
          W(S + RestoWs::sACC) = acc_count;
          W(S + RestoWs::sFLAST) = f_last;
          W(S + RestoWs::sSOFT) = soft ? 1.0 : 0.0;
          W(S + RestoWs::sSOFTN) = soft_count;
          W(S + RestoWs::sIT) = it;
          W(S + RestoWs::sSTEP) = step;
          W(S + RestoWs::sWARM) = warm ? 1.0 : 0.0;
          W(S + RestoWs::sTHK) = thk;
          W(S + RestoWs::sPHK) = phk;
          W(S + RestoWs::sGD) = gd;
          W(S + RestoWs::sAMAX) = amax;
          W(S + RestoWs::sAZ) = az;
          if (!sw_set) switching();
          W(S + RestoWs::sSWA) = sw_a;
          W(S + RestoWs::sACCNOW) = acceptable_now ? 1.0 : 0.0;
          W(S + RestoWs::sSOFTTRIED) = soft_tried ? 1.0 : 0.0;
          if constexpr (RESUME) {
            pending_rec = true;  // recovered at the top of the next pass
          } else {
            W(S + RestoWs::sPEND) = 1.0;  // left to the resume launch
            *a.park_flag = a.park_epoch;   // (vector store; every parking lane writes the same value)
            done = parked = true;
          }
          handled = true;
        }
      }
    }
    if (!done && !accepted && !handled) {
#ifdef MPCX_DEBUG_PRINT  // (not in the stamps build: its ISA is the product's, phase by phase)
      if (k == 0)
        printf("LSFAIL inst=%d step=%d it=%d mu=%.3e thk=%.6e phk=%.10e gd=%.3e amax=%.3e alpha=%.3e amin=%.3e "
               "node-0 Ed=%.3e Ec=%.3e Ecomp=%.3e E0=%.3e fs=%.3e dw=%.1e\n",
               inst, step, it, mu, thk, phk, gd, amax, alpha, amin, Ed, Ec, Ecomp0, E0, fs, delta);
#endif
      done = true;
      // IPOPT: "restoration phase called at an acceptable point" ends the solve at that point
      status = acceptable_now ? 1 : 3;
      its = it;
    }

    STAMP(7);
    phase();
    // ------------------------------------------------------------ update iterate
#ifdef MPCX_DEBUG_PRINT
    if (inst == 0 && k == 0 && !done && !handled)
      printf("STEP it=%d resto=0 alpha=%.17g alpha_d=%.17g ftype=%d mu=%.17g delta=%.3g thk=%.17g phk=%.17g\n", it, alpha,
             az, (int)ftype, mu, delta, thk, phk);
#endif
    if (!done && !handled) {
      if (!ftype && !soft_pd) {  // augment the filter (not after a soft step accepted by the pd error)
        if (filt.add((1.0 - kGammaTheta) * thk, phk - kGammaPhi * thk, k, xw)) DIAG(14);
      }
      // filter reset (IPOPT filter_reset_trigger = 5, max_filter_resets = 5): the filter is
      // cleared once the last rejection of 5 successive iterations was the filter's
      if (soft_pd) {
      } else if (lastrej_f) {
        if (++frej >= kFilterResetTrigger && nfreset < kMaxFilterResets) {
          filt.clear();
          ++nfreset;
          frej = 0;
          DIAG(9);
        }
      } else {
        frej = 0;
      }
#pragma unroll
      for (int i = 0; i < NZ; ++i) z[i] = fma(alpha, dz[i], z[i]);
#pragma unroll
      for (int i = 0; i < NX; ++i) lam[i] = fma(alpha, dlam[i], lam[i]);
      fresh = trial_fresh;
      lz_ok = acc0;  // z is the first trial point: its log-sum is Lt0
      Lz = Lt0;
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        if (hL[i]) {
          const double mrs = mu * rcp64(z[i] - lb[i]);
          zL[i] = fmax(fmin(zL[i] + az * dzL[i], kKappaSigma * mrs), mrs * (1.0 / kKappaSigma));
        }
        if (hU[i]) {
          const double mrs = mu * rcp64(ub[i] - z[i]);
          zU[i] = fmax(fmin(zU[i] + az * dzU[i], kKappaSigma * mrs), mrs * (1.0 / kKappaSigma));
        }
      }
    }
    STAMP(8);
    phase();
  }
  STAMP(9);
#ifdef MPCX_STAMPS
  if (g_mpcx_diag && valid && active && k == 0 && rho == 0)
    for (int i = 0; i < kDiag; ++i) g_mpcx_diag[(size_t)inst * kDiag + i] = diag[i];
  if (g_mpcx_stamps && !RESUME && (threadIdx.x & 63) == 0) {
    const long wv = gid / 64;
    for (int i = 0; i < kStampSlots; ++i) g_mpcx_stamps[wv * kStampSlots + i] = st_acc[i];
  }
#endif

  // ---- results (an instance that ended in a failed line search holds a trial's evaluation)
  if constexpr (Model::kEvalInSearch) {
    if (__any(!fresh))
      if (!fresh) sweep();
  }
  const double fsum = gsum<G>(hasU ? qv : 0.0, xw);
#ifdef MPCX_DEBUG_PRINT
  if (inst == 0 && (k % 64) == 0)
    printf("END k=%d fs=%g mu=%g it=%d lam0=%g z0=%g zL=%g zU=%g\n", k, fs, mu, it, lam[0], z[0], zL[NX], zU[NX]);
#endif
  const bool writes = valid && !parked && active && rho == 0;  // parked: the resume launch writes them
  if (writes) {
    double* w = a.w_out + (size_t)inst * nw;
    if (hasX)
      for (int i = 0; i < NX; ++i) w[ixw<NX, NU>(k, i)] = z[i];
    if (hasU)
      for (int i = 0; i < NU; ++i) w[iuw<NX, NU>(k, i)] = z[NX + i];
    if (a.lam_out && hasX)
      for (int i = 0; i < NX; ++i) a.lam_out[(size_t)inst * ng + NX * k + i] = lam[i] / fs;
    if (a.lamx_out) {
      double* lx = a.lamx_out + (size_t)inst * nw;
      if (hasX)
        for (int i = 0; i < NX; ++i) lx[ixw<NX, NU>(k, i)] = (zU[i] - zL[i]) / fs;
      if (hasU)
        for (int i = 0; i < NU; ++i) lx[iuw<NX, NU>(k, i)] = (zU[NX + i] - zL[NX + i]) / fs;
    }
    if (k == 0) {
      if (a.f_out) a.f_out[inst] = fsum;
      if (a.status) a.status[(size_t)step * a.B + inst] = status;
      if (a.iters) a.iters[(size_t)step * a.B + inst] = its;
    }
  }

  // ---- fused receding-horizon update (Casadi/multiple_shooting_casadi.py:271-287), the
  //      same result as shift_kernel: node k takes node k+1's primal and multipliers
  //      (last node / interval repeated), x0 <- F(x0, u_0*) on lane 0.
  if (a.w0_next) {  // kernel-uniform
    constexpr int NS = NZ + NX + NZ;  // z, lam, lamx of the next node
    double own[NS], nxt[NS];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      own[i] = z[i];
      own[NZ + NX + i] = (zU[i] - zL[i]) / fs;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) own[NZ + i] = lam[i] / fs;
    group_next<G, NS>(own, nxt, xw);
    if (writes) {
      const bool lastX = (k == N), lastU = (k == N - 1);
      double* w0n = a.w0_next + (size_t)inst * nw;
      if (hasX)
        for (int i = 0; i < NX; ++i) w0n[ixw<NX, NU>(k, i)] = lastX ? own[i] : nxt[i];
      if (hasU)
        for (int i = 0; i < NU; ++i) w0n[iuw<NX, NU>(k, i)] = lastU ? own[NX + i] : nxt[NX + i];
      if (a.lam0_next && hasX)
        for (int i = 0; i < NX; ++i) a.lam0_next[(size_t)inst * ng + NX * k + i] = lastX ? own[NZ + i] : nxt[NZ + i];
      if (a.lamx0_next) {
        double* lx = a.lamx0_next + (size_t)inst * nw;
        if (hasX)
          for (int i = 0; i < NX; ++i)
            lx[ixw<NX, NU>(k, i)] = k == 0 ? 0.0 : (lastX ? own[NZ + NX + i] : nxt[NZ + NX + i]);
        if (hasU)
          for (int i = 0; i < NU; ++i)
            lx[iuw<NX, NU>(k, i)] = lastU ? own[NZ + NX + NX + i] : nxt[NZ + NX + NX + i];
      }
      if (k == 0) {  // plant: x0 <- F(x0, u_0*) with the stage-0 model
        double zp[NZ], xfp[NX], qp;
#pragma unroll
        for (int i = 0; i < NX; ++i) zp[i] = x0[i];
#pragma unroll
        for (int i = 0; i < NU; ++i) zp[NX + i] = z[NX + i];
        Model::value(ma, ctx, zp, xfp, qp);
        double* pn = a.P_next + (size_t)inst * a.p_stride;
        for (int i = 0; i < NX; ++i) pn[i] = xfp[i];
      }
    }
  }
}

// Plant: x+ = F(x0, u) (Casadi/multiple_shooting_casadi.py:273), one thread per instance.
template <class Model>
__global__ void plant_kernel(SolveArgs a, const double* __restrict__ U, double* __restrict__ XF,
                             double* __restrict__ QF) {
  constexpr int NX = Model::NX, NU = Model::NU;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const double* p = a.P + (size_t)b * a.p_stride;
  const ModelArgs ma = model_args(a);
  typename Model::Ctx ctx;
  Model::load_ctx(ma, b, p, 0, true, ctx);
  double z[NX + NU], xf[NX], q;
  for (int i = 0; i < NX; ++i) z[i] = p[i];
  for (int i = 0; i < NU; ++i) z[NX + i] = U[(size_t)b * NU + i];
  Model::value(ma, ctx, z, xf, q);
  for (int i = 0; i < NX; ++i) XF[(size_t)b * NX + i] = xf[i];
  if (QF) QF[b] = q;
}

// Closed-loop update (:271-287): x0 <- F(x0, u0*), w0_next = w shifted one interval;
// multipliers shifted alike when given (warm start of the next solve).
template <class Model>
__global__ void shift_kernel(SolveArgs a, double* __restrict__ P, const double* __restrict__ W,
                             double* __restrict__ W0, const double* __restrict__ L, double* __restrict__ L0,
                             const double* __restrict__ LX, double* __restrict__ LX0) {
  constexpr int NX = Model::NX, NU = Model::NU, NZ = NX + NU;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int N = a.N, nw = NX + NZ * N, ng = NX * (N + 1);
  double* p = P + (size_t)b * a.p_stride;
  const double* w = W + (size_t)b * nw;
  double* w0 = W0 + (size_t)b * nw;
  const ModelArgs ma = model_args(a);
  typename Model::Ctx ctx;
  Model::load_ctx(ma, b, p, 0, true, ctx);
  double z[NZ], xf[NX], q;
  for (int i = 0; i < NX; ++i) z[i] = p[i];
  for (int i = 0; i < NU; ++i) z[NX + i] = w[iuw<NX, NU>(0, i)];
  Model::value(ma, ctx, z, xf, q);
  for (int i = 0; i < NX; ++i) p[i] = xf[i];
  // shifted guess: X_k <- X_{k+1}, U_k <- U_{k+1}; last node/interval repeated
  for (int kk = 0; kk <= N; ++kk) {
    const int src = kk < N ? kk + 1 : N;
    for (int i = 0; i < NX; ++i) w0[ixw<NX, NU>(kk, i)] = w[ixw<NX, NU>(src, i)];
    if (LX && LX0)
      for (int i = 0; i < NX; ++i)
        LX0[(size_t)b * nw + ixw<NX, NU>(kk, i)] = kk == 0 ? 0.0 : LX[(size_t)b * nw + ixw<NX, NU>(src, i)];
    if (L && L0)
      for (int i = 0; i < NX; ++i) L0[(size_t)b * ng + NX * kk + i] = L[(size_t)b * ng + NX * src + i];
    if (kk < N) {
      const int su = kk + 1 < N ? kk + 1 : N - 1;
      for (int i = 0; i < NU; ++i) w0[iuw<NX, NU>(kk, i)] = w[iuw<NX, NU>(su, i)];
      if (LX && LX0)
        for (int i = 0; i < NU; ++i) LX0[(size_t)b * nw + iuw<NX, NU>(kk, i)] = LX[(size_t)b * nw + iuw<NX, NU>(su, i)];
    }
  }
}

// Constraint values g = [x0 - X_0; F(X~_k, U_k) - X_{k+1}] with X~_0 = x0 and X~_k = X_k for k >= 1
// (Casadi/multiple_shooting_casadi.py:125,131,157,172-175: interval 0 integrates from the parameter).
template <class Model>
__global__ void constraints_kernel(SolveArgs a, const double* __restrict__ W, double* __restrict__ Gout) {
  constexpr int NX = Model::NX, NU = Model::NU, NZ = NX + NU;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int N = a.N, nw = NX + NZ * N, ng = NX * (N + 1);
  const double* p = a.P + (size_t)b * a.p_stride;
  const double* w = W + (size_t)b * nw;
  double* g = Gout + (size_t)b * ng;
  for (int i = 0; i < NX; ++i) g[i] = p[i] - w[i];
  const ModelArgs ma = model_args(a);
  for (int kk = 0; kk < N; ++kk) {
    typename Model::Ctx ctx;
    Model::load_ctx(ma, b, p, kk, true, ctx);
    double z[NZ], xf[NX], q;
    for (int i = 0; i < NX; ++i) z[i] = kk == 0 ? p[i] : w[ixw<NX, NU>(kk, i)];
    for (int i = 0; i < NU; ++i) z[NX + i] = w[iuw<NX, NU>(kk, i)];
    Model::value(ma, ctx, z, xf, q);
    for (int i = 0; i < NX; ++i) g[NX * (kk + 1) + i] = xf[i] - w[ixw<NX, NU>(kk + 1, i)];
  }
}

// ---- launch helpers (called from capi.cpp) -----------------------------------
// The solve kernel instantiation a launch picks: G lanes per group, R replicas of it per wave.  A
// 32-lane group widened to a wave runs replicated (R = 2) where the model has that instantiation;
// the results are the same bits either way (models.h stage_derivs).
template <class Model>
static void solve_shape(const SolveArgs& a, int* G, int* R) {
  *G = solve_group_size(a.N, a.B, a.n_simd, a.group_policy);
  *R = 1;
  if constexpr (ReplicateOf<Model>::value) {
    const int narrow = solve_group_size(a.N, a.B, a.n_simd, 1);
    if (*G == 64 && narrow == 32) {
      *G = 32;
      *R = 2;
    }
    // a replicating model's 32-lane kernel sums the evaluation moments in the replicas' two halves
    // (models.h stage_derivs); a 16-lane group (N < 16) sums them in one pass at 16 and 64 lanes, so
    // it is never widened to exactly 32 lanes, where its bits would follow the halves' order
    if (narrow == 16 && *G == 32) *G = 16;
  }
}

template <class Model>
static hipError_t launch_solve_model(const SolveArgs& a, hipStream_t stream) {
  // lane group: the smallest power of two holding nodes 0..N; G > 64 spans G/64 waves.
  // A batch too small to give every SIMD a wave gets wider groups (up to one instance per
  // wave): the per-wave instruction stream is the same, but a wave then runs only its own
  // instance's iterations, not the maximum over the instances it holds (config 2: +5 %
  // solves/s in multi-step launches).  spec.group_policy = 1 keeps the narrowest group.
  // (Measured and not adopted: collectives over the 32 lanes of config 2's nodes on the same
  // 64-lane grid -- no gain)
  int Gk, R;
  solve_shape<Model>(a, &Gk, &R);
  const int G = Gk * R;  // lanes per instance on the grid
  const long threads = (long)a.B * G;
  const int bs = G > 64 ? G : 64;
  const int blocks = (int)((threads + bs - 1) / bs);
  if constexpr (ReplicateOf<Model>::value)
    if (R == 2) {
      hipLaunchKernelGGL((solve_kernel<Model, 32, false, 2>), dim3(blocks), dim3(64), 0, stream, a);
      return hipGetLastError();
    }
  if (G == 16) hipLaunchKernelGGL((solve_kernel<Model, 16>), dim3(blocks), dim3(64), 0, stream, a);
  else if (G == 32) hipLaunchKernelGGL((solve_kernel<Model, 32>), dim3(blocks), dim3(64), 0, stream, a);
  else if (G == 64) hipLaunchKernelGGL((solve_kernel<Model, 64>), dim3(blocks), dim3(64), 0, stream, a);
  else if (G == 128) hipLaunchKernelGGL((solve_kernel<Model, 128>), dim3(blocks), dim3(128), 0, stream, a);
  else hipLaunchKernelGGL((solve_kernel<Model, 256>), dim3(blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// the resume launch (models with a restoration phase): same grid, the parked groups only
template <class Model>
static hipError_t launch_resume_model(const SolveArgs& a, hipStream_t stream) {
  if constexpr (!RestoOf<Model>::value) {
    return hipSuccess;
  } else {
    int Gk, R;
    solve_shape<Model>(a, &Gk, &R);
    const int G = Gk * R;
    const long threads = (long)a.B * G;
    const int bs = G > 64 ? G : 64;
    const int blocks = (int)((threads + bs - 1) / bs);
    if constexpr (ReplicateOf<Model>::value)
      if (R == 2) {
        hipLaunchKernelGGL((solve_kernel<Model, 32, true, 2>), dim3(blocks), dim3(64), 0, stream, a);
        return hipGetLastError();
      }
    if (G == 16) hipLaunchKernelGGL((solve_kernel<Model, 16, true>), dim3(blocks), dim3(64), 0, stream, a);
    else if (G == 32) hipLaunchKernelGGL((solve_kernel<Model, 32, true>), dim3(blocks), dim3(64), 0, stream, a);
    else if (G == 64) hipLaunchKernelGGL((solve_kernel<Model, 64, true>), dim3(blocks), dim3(64), 0, stream, a);
    else if (G == 128) hipLaunchKernelGGL((solve_kernel<Model, 128, true>), dim3(blocks), dim3(128), 0, stream, a);
    else hipLaunchKernelGGL((solve_kernel<Model, 256, true>), dim3(blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
  }
}

template <class Model>
static hipError_t launch_plant_model(const SolveArgs& a, const double* U, double* XF, double* QF, hipStream_t stream) {
  hipLaunchKernelGGL((plant_kernel<Model>), dim3((a.B + 255) / 256), dim3(256), 0, stream, a, U, XF, QF);
  return hipGetLastError();
}

template <class Model>
static hipError_t launch_constraints_model(const SolveArgs& a, const double* W, double* Gout, hipStream_t stream) {
  hipLaunchKernelGGL((constraints_kernel<Model>), dim3((a.B + 255) / 256), dim3(256), 0, stream, a, W, Gout);
  return hipGetLastError();
}

template <class Model>
static hipError_t launch_shift_model(const SolveArgs& a, double* P, const double* W, double* W0, const double* L,
                                     double* L0, const double* LX, double* LX0, hipStream_t stream) {
  hipLaunchKernelGGL((shift_kernel<Model>), dim3((a.B + 255) / 256), dim3(256), 0, stream, a, P, W, W0, L, L0, LX,
                     LX0);
  return hipGetLastError();
}

}  // namespace mpcx

// One translation unit per model: the launch entry points solver.hip dispatches to (and, in
// the diagnostic build, this unit's setters of its own copies of the stamp/counter pointers).
#ifdef MPCX_STAMPS
#define MPCX_INSTANTIATE_DIAG(tag)                                                      \
  int diag_set_stamps_##tag(void* d) {                                                  \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_mpcx_stamps), &d, sizeof(void*));        \
  }                                                                                     \
  int diag_set_counters_##tag(void* d) {                                                \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_mpcx_diag), &d, sizeof(void*));          \
  }
#else
#define MPCX_INSTANTIATE_DIAG(tag)
#endif
#define MPCX_INSTANTIATE(Model, tag, name)                                                                  \
  namespace mpcx {                                                                                          \
  hipError_t solve_shape_##tag(const SolveArgs& a, int* G, int* R, const char** kname) {                     \
    solve_shape<Model>(a, G, R);                                                                            \
    *kname = name;                                                                                          \
    return hipSuccess;                                                                                      \
  }                                                                                                         \
  hipError_t launch_solve_##tag(const SolveArgs& a, hipStream_t s) { return launch_solve_model<Model>(a, s); } \
  hipError_t launch_resume_##tag(const SolveArgs& a, hipStream_t s) { return launch_resume_model<Model>(a, s); } \
  hipError_t launch_plant_##tag(const SolveArgs& a, const double* U, double* XF, double* QF, hipStream_t s) {   \
    return launch_plant_model<Model>(a, U, XF, QF, s);                                                      \
  }                                                                                                         \
  hipError_t launch_constraints_##tag(const SolveArgs& a, const double* W, double* Gout, hipStream_t s) {      \
    return launch_constraints_model<Model>(a, W, Gout, s);                                                  \
  }                                                                                                         \
  hipError_t launch_shift_##tag(const SolveArgs& a, double* P, const double* W, double* W0, const double* L,  \
                                double* L0, const double* LX, double* LX0, hipStream_t s) {                 \
    return launch_shift_model<Model>(a, P, W, W0, L, L0, LX, LX0, s);                                       \
  }                                                                                                         \
  MPCX_INSTANTIATE_DIAG(tag)                                                                                \
  }
