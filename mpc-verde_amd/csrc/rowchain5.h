// rowchain5.h -- the 5-state, one-input linear model's full Riccati steps spread over a 16-lane row
// (gfx950 device code; DESIGN.md §3.1 "row chain"): config 5's cart-pole QP, whose decoupled suffix
// the vector scan handles, leaves a short chain of full steps (the free moves, nodes 0 .. kb - 1)
// on wave 0 of its two-wave group.  The same step as riccati.h riccati_step<5, 1, dense, dense,
// DEC = false, SREORD = true> -- the same operations in the same order, so the same bits, signs of
// exact zeros included (the model's A has an all-zero column) -- with every row lane owning one
// COLUMN of the step's products:
//
//   row lane   0 .. 4      5 6 7     8    9 10 11    12    13 14 15
//   column     x0 .. x4    (dummy)   s    (dummy)    u     (dummy)
//
// (s: P c + p on the value-function side, the gradient on the stage side; s and u in DPP banks 2
// and 3 of their own, so a bank-masked FMA adds p on lane s alone).  A step:
//   stage 1  V_b = P W_b, W_b = column b of [A c B], every sum product-first (an FMA into -0.0 is
//            the product, sign of zero included); lane s then adds p (riccati.h SREORD)
//   stage 2  Q_{ib} = H_{ib} + sum_m A_{mi} V_{mb} (Hxx' on the x lanes, gx on lane s) and
//            U_b = H_{ub} + sum_m B_m V_{mb} (Hux' as B^T (P A) on the x lanes -- riccati.h's order
//            for dense A and B -- Huu' on lane u, gu on lane s)
//   factor   r0 = 1 / Huu' (every lane, one broadcast)
//   update   P_k(i, c) = Hxx'(i, c) - (r0 h0_i) h0_c on lane c, p_k on lane s
// ≈ 75 VALU instructions where riccati_step issues ≈ 400 for one lane.  Stage data reach the rows
// through LDS node records (one 12-double block per column: H column, then W) that the node lanes
// write before the chain; after step j row 0's x and s lanes store P_j's columns, p_j and the
// step's factors (h0_c, g0, r0, d0) into node j's consumed record, and node lane k reads its own
// back -- no step is redone.  tests/hip/rowchain_check.hip compares the chain with the sequential
// recursion bit for bit.
#pragma once
#include <hip/hip_runtime.h>

#include "collectives.h"
#include "riccati.h"
#include "rowchain.h"

namespace mpcx {

namespace rowchain5 {

constexpr int NX = 5, NU = 1, NZ = NX + NU;
constexpr int kBlk = 12;               // doubles per column block: H rows x0..x4, u; W rows 0..4; pad
constexpr int kNB = NX + 2;            // blocks per node: x0..x4, s, u
constexpr int kBS = NX, kBU = NX + 1;  // blocks of s and u
constexpr int kRec = kBlk * kNB + 2;   // 86 doubles per node record (the pad staggers LDS banks)
constexpr int kLS = 8, kLU = 12;       // lanes of s and u (x_c on lane c)
constexpr int kMax = 8;                // longest chain (records kMax + 1: node jc's value function)

// the structure the chain hard-codes: dense A and B, no declared unit entries, Hux' as B^T (P A)
template <class Model>
constexpr bool fits() {
  if constexpr (Model::NX != NX || Model::NU != NU) {
    return false;
  } else {
    return Model::AMASK == (1ull << (NX * NX)) - 1 && Model::BMASK == (1ull << (NX * NU)) - 1 &&
           AOneOf<Model>::value == 0 && !hux_by_atpb<NX, NU, Model::AMASK, Model::BMASK>();
  }
}

// node k's stage into its record (node lane k below the chain's top)
__device__ __forceinline__ void store_node(double* rk, const double* Hd, const double* gp, const double* A,
                                           const double* Bm, const double* c) {
  typedef double v2d __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int b = 0; b < kNB; ++b) {
    double v[kBlk];
#pragma unroll
    for (int i = 0; i < NZ; ++i) v[i] = b == kBS ? gp[i] : Hd[symix(i, b == kBU ? NX : b, NZ)];
#pragma unroll
    for (int m = 0; m < NX; ++m) v[NZ + m] = b < NX ? A[m * NX + b] : b == kBS ? c[m] : Bm[m];
    v[kBlk - 1] = 0.0;
#pragma unroll
    for (int q = 0; q < kBlk / 2; ++q) *reinterpret_cast<v2d*>(rk + b * kBlk + 2 * q) = v2d{v[2 * q], v[2 * q + 1]};
  }
}

// the chain's start, node jc's value function (P_jc upper triangle, p_jc), as columns; zeros on the
// u lane (its stage-1 start is multiplied by nothing, but a non-finite value must not reach it)
__device__ __forceinline__ void store_terminal(double* rk, const double* P, const double* p) {
#pragma unroll
  for (int b = 0; b < kNB; ++b)
#pragma unroll
    for (int i = 0; i < NX; ++i) rk[b * kBlk + i] = b < NX ? P[symix(i, b, NX)] : b == kBS ? p[i] : 0.0;
}

// node k's results after the chain (its own record): P_k, p_k, the factors riccati_step would leave
// (NU = 1: t, r1, h1, g1 zero) and its verdict d0 > 0
__device__ __forceinline__ bool load_result(const double* rk, double* P, double* p, Fac<NX, NU>& f) {
#pragma unroll
  for (int j = 0; j < NX; ++j) {
#pragma unroll
    for (int i = 0; i <= j; ++i) P[symix(i, j, NX)] = rk[j * kBlk + i];
    f.h0[j] = rk[j * kBlk + NX];
    f.h1[j] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) p[i] = rk[kBS * kBlk + i];
  f.g0 = rk[kBS * kBlk + NX];
  f.r0 = rk[NX + 1];
  f.r1 = 0.0;
  f.t = 0.0;
  f.g1 = 0.0;
  return rk[kBS * kBlk + NX + 2] > 0.0;
}

// The chain: steps jc - 1 .. 0 over the records at `rec` (node 0's; node jc's holds the start).  One
// instance per wave: every lane of the wave runs it (a broadcast source must be active), row 0 stores.
// Each group of DPP FMAs is one asm statement whose DPP sources are LDS loads or were written at
// least two wait states earlier (the VALU-write -> DPP-read hazard the compiler does not see inside
// the asm).
__device__ __forceinline__ void run(double* rec, int jc) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  // lane constants, derived inside the solve loop (opaque to loop-invariant code motion)
  int r = (int)(threadIdx.x & 15);
  asm volatile("" : "+v"(r));
  const int blk = r < NX ? r : r == kLU ? kBU : kBS;  // dummies read block s
  double negz = -0.0, one = 1.0;
  asm volatile("" : "+v"(negz), "+v"(one));
  const unsigned long long wmask = __ballot((threadIdx.x & 63) < 16 && (r < NX || r == kLS));
  double* bp = rec + blk * kBlk;  // this lane's block of node 0
  struct Stage {
    v2d L[kBlk / 2];
  };
  auto load = [&](int j) __attribute__((always_inline)) {
    const double* q = bp + j * kRec;
    Stage s;
#pragma unroll
    for (int i = 0; i < kBlk / 2; ++i) s.L[i] = *reinterpret_cast<const v2d*>(q + 2 * i);
    return s;
  };
  struct Out {
    double* o;
    double s[NX];
    double u, r0, d0;
  };
  // row 0's x and s lanes store under their exec mask, no branch; the node lanes read these records
  // after the chain from the same wave (LDS operations complete in order)
  auto store = [&](const Out& o) __attribute__((always_inline)) {
    const unsigned a = (unsigned)(unsigned long)((__attribute__((address_space(3))) double*)o.o);
    unsigned long long saved;
    asm volatile(
        "s_and_saveexec_b64 %0, %1\n\t"
        "ds_write2_b64 %2, %3, %4 offset1:1\n\t"
        "ds_write2_b64 %2, %5, %6 offset0:2 offset1:3\n\t"
        "ds_write2_b64 %2, %7, %8 offset0:4 offset1:5\n\t"
        "ds_write2_b64 %2, %9, %10 offset0:6 offset1:7\n\t"
        "s_or_b64 exec, exec, %0"
        : "=&s"(saved)
        : "s"(wmask), "v"(a), "v"(o.s[0]), "v"(o.s[1]), "v"(o.s[2]), "v"(o.s[3]), "v"(o.s[4]), "v"(o.u),
          "v"(o.r0), "v"(o.d0)
        : "memory", "scc");  // (the exec save / restore sets SCC)
  };
  double S0, S1, S2, S3, S4;
  {
    const double* t = bp + jc * kRec;
    S0 = t[0], S1 = t[1], S2 = t[2], S3 = t[3], S4 = t[4];
  }
  // one step: its record loaded at the step's start and its results stored at its end -- no
  // prefetch, no deferred store, no second register set: the chain is a few steps long, and the
  // registers the overlap would hold are the ones the rest of the solve loop spills first (a
  // prefetching, double-buffered chain measured slower on config 5 for its spills elsewhere)
  auto step = [&](int j) __attribute__((always_inline)) {
    const Stage st = load(j);
    const double W0 = st.L[3].x, W1 = st.L[3].y, W2 = st.L[4].x, W3 = st.L[4].y, W4 = st.L[5].x;
    // ---- stage 1: V_r = sum_m P_{rm} w_m product-first (into -0.0), then + p_r on lane s.  The five
    // start moves put any earlier VALU write of S two instructions back
    double V0, V1, V2, V3, V4;
    asm volatile(
        "v_mov_b64 %0, %15\n\t"
        "v_mov_b64 %1, %15\n\t"
        "v_mov_b64 %2, %15\n\t"
        "v_mov_b64 %3, %15\n\t"
        "v_mov_b64 %4, %15\n\t"
        "v_fmac_f64_dpp %0, %5, %10 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %5, %10 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %5, %10 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %5, %10 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %5, %10 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %5, %11 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %6, %11 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %6, %11 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %6, %11 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %6, %11 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %5, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %6, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %7, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %7, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %7, %12 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %5, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %6, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %7, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %8, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %5, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %6, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %7, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %9, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %5, %16 row_newbcast:8 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %1, %6, %16 row_newbcast:8 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %2, %7, %16 row_newbcast:8 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %3, %8, %16 row_newbcast:8 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %4, %9, %16 row_newbcast:8 row_mask:0xf bank_mask:0x4"
        : "=&v"(V0), "=&v"(V1), "=&v"(V2), "=&v"(V3), "=&v"(V4)
        : "v"(S0), "v"(S1), "v"(S2), "v"(S3), "v"(S4), "v"(W0), "v"(W1), "v"(W2), "v"(W3), "v"(W4), "v"(negz),
          "v"(one));
    // ---- stage 2: the x rows and the u row (B^T (P A) on the x lanes).  The s_nop covers a register
    // copy of a W the compiler might place just before the block
    double Q0 = st.L[0].x, Q1 = st.L[0].y, Q2 = st.L[1].x, Q3 = st.L[1].y, Q4 = st.L[2].x, U = st.L[2].y;
    asm volatile(
        "s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %11, %6 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %11, %6 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %11, %6 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %11, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %11, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %11, %6 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %12, %7 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %12, %7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %12, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %12, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %12, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %12, %7 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %13, %8 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %13, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %13, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %13, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %13, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %13, %8 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %14, %9 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %14, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %14, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %14, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %14, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %14, %9 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %15, %10 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %15, %10 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %15, %10 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %15, %10 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %15, %10 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %15, %10 row_newbcast:12 row_mask:0xf bank_mask:0xf"
        : "+v"(Q0), "+v"(Q1), "+v"(Q2), "+v"(Q3), "+v"(Q4), "+v"(U)
        : "v"(V0), "v"(V1), "v"(V2), "v"(V3), "v"(V4), "v"(W0), "v"(W1), "v"(W2), "v"(W3), "v"(W4));
    // ---- factor: Huu' on lane u, every lane
    const double d0 = rowchain::bcast<kLU>(U);
    const double r0 = rcp64(d0);
    // ---- update: P_k(i, c) = Hxx'(i, c) - (r0 h0_i) h0_c, (r0 h)_i from lane x_i; h0_c = U (lane s:
    // gu).  One s_nop between R0's write and its first DPP read
    double R0;
    asm volatile(
        "v_mul_f64 %5, %6, %7\n\t"
        "s_nop 1\n\t"
        "v_fmac_f64_dpp %0, -%5, %7 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%5, %7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, -%5, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, -%5, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, -%5, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf"
        : "+v"(Q0), "+v"(Q1), "+v"(Q2), "+v"(Q3), "+v"(Q4), "=&v"(R0)
        : "v"(r0), "v"(U));
    S0 = Q0, S1 = Q1, S2 = Q2, S3 = Q3, S4 = Q4;
    store(Out{bp + j * kRec, {S0, S1, S2, S3, S4}, U, r0, d0});
  };
  for (int j = jc - 1; j >= 0; --j) step(j);
}

}  // namespace rowchain5

}  // namespace mpcx
