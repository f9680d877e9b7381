// rowchain6.h -- the 6-state bicycle's backward Riccati recursion spread over 16-lane rows
// (gfx950 device code; DESIGN.md §3.1 "row chain").  The unicycle's row chain (rowchain.h) widened
// to NX = 6: the same step as riccati.h riccati_step for the model's Jacobian structure -- the same
// operations in the same order, so the same bits -- with every lane of a 16-lane row owning one
// COLUMN of the step's products:
//
//   row lane   0 .. 5      6  7    8   9   10    11 .. 15
//   column     x0 .. x5    (dummy) s   u0  u1    (dummy)
//
// The x lanes sit in DPP banks 0-1 and the s and u lanes in bank 2, so one accumulator per lane
// serves both sums that differ between them (bank-masked DPP FMAs, below).  Operands another lane
// owns arrive as the row_newbcast source of a v_fmac_f64_dpp.  A step:
//   stage 1  V_b = P W_b (+ p on lane s), W_b = column b of [A c B] (36 FMAs; P_{rm} from lane
//            max(r, m), register min(r, m): lane c keeps column c of P, lane s keeps p)
//   stage 2  Q_{ib} = H_{ib} + sum_m A_{mi} V_{mb}, i = x0..x5 (A's structural zeros skipped:
//            columns x0, x1 of A are unit vectors) -- Hxx' on the x lanes, gx on lane s;
//            U_{lb} = H_{u_l b} + sum_m B_{ml} V_{mb} on lanes s, u (Huu', gu) and
//            U_{lc} = H_{u_l c} + sum_m (P B)_{ml} A_{mc} on the x lanes (Hux' as riccati.h's
//            A^T (P B), the order its kAtPB rule picks for this model)
//   factor   the 2x2 L D L^T of Huu' (every lane, from three broadcasts)
//   update   P_k(i, c) = Hxx'(i, c) - (r0 h0_i) h0_c - (r1 h1_i) h1_c on lane c, p_k on lane s
// about 130 VALU instructions where riccati_step issues about 680 for one lane.  Every row runs
// the instance's whole chain (one instance per 64-lane wave: four identical rows).
//
// Stage data reach the rows through LDS node records -- one 14-double block per column: H column
// (x rows, u rows), then W -- that the node lanes write before the steps that read them.  A
// record is 1 KB, so the LDS holds a window of kWin nodes at a time (the ring aliases the
// stage evaluations' transcendental cache, idle here): the chain runs window by window, the node
// lanes of the next window refilling the ring in between.  The chain hands back only the value
// functions (row 0's x and s lanes store P_j's columns and p_j to global memory, node j's slots);
// afterwards node lane k redoes its own step from node k+1's value function -- riccati_step, all
// nodes at once -- for its factors and P_k.  tests/hip/rowchain_check.hip compares the chain with
// the sequential recursion bit for bit.
#pragma once
#include <hip/hip_runtime.h>

#include "collectives.h"
#include "riccati.h"
#include "rowchain.h"

namespace mpcx {

namespace rowchain6 {

constexpr int NX = 6, NU = 2, NZ = NX + NU;
constexpr int kBlk = 14;               // doubles per column block: H rows x0..x5, u0, u1; W rows 0..5
constexpr int kNB = NX + 1 + NU;       // blocks per node: x0..x5, s, u0, u1
constexpr int kRec = kBlk * kNB;       // 126 doubles per node record (16-byte aligned blocks)
constexpr int kLS = 8, kLU0 = 9, kLU1 = 10;  // lanes of s, u0, u1 (x_c on lane c)
constexpr int kOut = (NX + 1) * NX;    // per node output: P_j's columns x0..x5, then p_j
constexpr int kWin = 35;               // nodes per window: (kWin + 1) records in the ring (+ node N)
constexpr int kRing = (kWin + 1) * kRec;

// the structure the chain hard-codes: columns x0, x1 of A are e0, e1 (f does not read X, Y), the
// other columns dense, B dense, no declared unit entries, Hux' as A^T (P B)
__host__ __device__ constexpr unsigned long long amask6() {
  unsigned long long m = 0;
  for (int r = 0; r < NX; ++r)
    for (int j = 0; j < NX; ++j)
      if (j >= 2 || r == j) m |= 1ull << (r * NX + j);
  return m;
}
template <class Model>
constexpr bool fits() {
  if constexpr (Model::NX != NX || Model::NU != NU) {
    return false;
  } else {
    return Model::AMASK == amask6() && Model::BMASK == (1ull << (NX * NU)) - 1 && AOneOf<Model>::value == 0 &&
           hux_by_atpb<NX, NU, Model::AMASK, Model::BMASK>();
  }
}

// node k's stage into its record (node lane k < N): Hd = Hs + diag(Sigma + delta) (the kernel's
// order of that sum), gradient gp, defect c, Jacobians A, B (structural zeros as zeros)
__device__ __forceinline__ void store_node(double* rk, const double* Hs, const double* sig, double delta,
                                           const double* A, const double* Bm, const double* gp, const double* c) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  auto Hd = [&](int i, int j) __attribute__((always_inline)) {
    double h = Hs[symix(i, j, NZ)];
    if (i == j) h += sig[i] + delta;
    return h;
  };
#pragma unroll
  for (int b = 0; b < kNB; ++b) {
    double v[kBlk];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      if (b < NX) v[i] = i < NX ? Hd(i, b) : Hd(b, i);  // x_b: H(i, x_b), H(u_l, x_b)
      else if (b == NX) v[i] = gp[i];                    // s: the gradient
      else v[i] = Hd(i, b - 1);                          // u_l: H(i, u_l) (z index NX + l = b - 1)
    }
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      if (b < NX) v[NZ + m] = (amask6() >> (m * NX + b)) & 1ull ? A[m * NX + b] : 0.0;
      else if (b == NX) v[NZ + m] = c[m];
      else v[NZ + m] = Bm[m * NU + (b - NX - 1)];
    }
#pragma unroll
    for (int q = 0; q < kBlk / 2; ++q) *reinterpret_cast<v2d*>(rk + b * kBlk + 2 * q) = v2d{v[2 * q], v[2 * q + 1]};
  }
}

// node N's value function, the chain's start (in the first kBlk slots' H rows of a record):
// P_N = diag(Sigma_x + delta) on the x lanes, p_N = gradient on lane s, zeros on the u lanes (their
// stage-1 start is multiplied by 0, which must not meet an inf or NaN)
__device__ __forceinline__ void store_terminal(double* rk, const double* sig, double delta, const double* gp) {
#pragma unroll
  for (int b = 0; b < kNB; ++b)
#pragma unroll
    for (int i = 0; i < NX; ++i)
      rk[b * kBlk + i] = b < NX ? (i == b ? sig[b] + delta : 0.0) : b == NX ? gp[i] : 0.0;
}

// node k+1's value function after the chain (node lane k < N reads node k+1's output slots): the
// operands of its own riccati_step, as the sequential recursion hands them on
__device__ __forceinline__ void load_next(const double* o, double* P, double* p) {
#pragma unroll
  for (int j = 0; j < NX; ++j)
#pragma unroll
    for (int i = 0; i <= j; ++i) P[symix(i, j, NX)] = ((const __attribute__((address_space(1))) double*)o)[j * NX + i];
#pragma unroll
  for (int i = 0; i < NX; ++i) p[i] = ((const __attribute__((address_space(1))) double*)o)[NX * NX + i];
}

// The chain: steps N-1 .. 0, window by window.  Every lane of the wave runs it (a broadcast source
// must be active).  `ring` = this wave's LDS ring, `out0` = node 0's output slots (global; node j's
// at out0 + j * ostride), `writer` = this wave's outputs are kept (a valid instance).  `fill(lo, hi,
// top)` is run by the whole wave before the steps of nodes lo..hi: node lanes lo..hi write their
// records to ring slots k - lo, and with `top` node N's lane its value function to slot N - lo.
// Each group of DPP FMAs is one asm statement whose DPP sources are LDS loads or were written at
// least two VALU instructions earlier (the VALU-write -> DPP-read hazard the compiler does not
// see inside the asm).
// Returns true when the chain stopped early: a step whose reduced Huu' is not positive definite
// (fac_ok of its factors false) decides the inertia-correction attempt, so the chain ends there (every
// lane holds the step's reciprocals; the four rows agree: a wave-uniform exit).
template <class Fill>
__device__ __forceinline__ bool run(double* ring, double* out0, long ostride, bool writer, int N, Fill&& fill) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  // lane constants, derived inside the solve loop (opaque to loop-invariant code motion)
  int r = (int)(threadIdx.x & 15);
  asm volatile("" : "+v"(r));
  const int blk = r < NX ? r : r == kLU0 ? NX + 1 : r == kLU1 ? NX + 2 : NX;  // dummies read block s
  const double m_s = r == kLS ? 1.0 : 0.0;
  const unsigned long long wmask = __ballot(writer && (threadIdx.x & 63) < 16 && (r < NX || r == kLS));
  double* op = out0 + (r < NX ? r : NX) * NX;  // this lane's column of node 0's output
  const double* bp = ring + blk * kBlk;        // this lane's block of ring slot 0
  struct Stage {
    v2d L[kBlk / 2];
  };
  auto load = [&](int slot) __attribute__((always_inline)) {
    const double* q = bp + slot * kRec;
    Stage s;
#pragma unroll
    for (int i = 0; i < kBlk / 2; ++i) s.L[i] = *reinterpret_cast<const v2d*>(q + 2 * i);
    return s;
  };
  struct Out {
    double* o;
    double s[NX];
  };
  // row 0's x and s lanes store (the other rows hold the same bits), under their exec mask, no
  // branch.  Nothing reads these stores before the chain ends (the caller's barrier).
  auto store = [&](const Out& o) __attribute__((always_inline)) {
    unsigned long long saved;
    asm volatile(
        "s_and_saveexec_b64 %0, %1\n\t"
        "global_store_dwordx2 %2, %3, off\n\t"
        "global_store_dwordx2 %2, %4, off offset:8\n\t"
        "global_store_dwordx2 %2, %5, off offset:16\n\t"
        "global_store_dwordx2 %2, %6, off offset:24\n\t"
        "global_store_dwordx2 %2, %7, off offset:32\n\t"
        "global_store_dwordx2 %2, %8, off offset:40\n\t"
        "s_or_b64 exec, exec, %0"
        : "=&s"(saved)
        : "s"(wmask), "v"(o.o), "v"(o.s[0]), "v"(o.s[1]), "v"(o.s[2]), "v"(o.s[3]), "v"(o.s[4]), "v"(o.s[5])
        : "scc");  // (the exec save / restore sets SCC)
  };

  int lo = N > kWin ? N - kWin : 0, hi = N - 1;
  asm volatile("" ::: "memory");
  fill(lo, hi, true);
  asm volatile("" ::: "memory");
  double S0, S1, S2, S3, S4, S5;
  {
    const double* t = bp + (N - lo) * kRec;
    S0 = t[0], S1 = t[1], S2 = t[2], S3 = t[3], S4 = t[4], S5 = t[5];
  }
  Out oa{op + (long)N * ostride, {S0, S1, S2, S3, S4, S5}}, ob;  // node N's (stored during step N - 1)
  // one step on the loaded stage `st`, the next record's loads into `nx`, the previous step's
  // results `po` stored and this step's in `no`; true = the step fails the inertia test.  Two stage
  // and two result variables alternate between steps (pairs of steps below): one loop-carried set
  // would cost register copies at every back edge
  auto step = [&](int j, const Stage& st, Stage& nx, const Out& po, Out& no) __attribute__((always_inline)) {
    const double H0 = st.L[0].x, H1 = st.L[0].y, H2 = st.L[1].x, H3 = st.L[1].y, H4 = st.L[2].x,
                 H5 = st.L[2].y;
    const double W0 = st.L[4].x, W1 = st.L[4].y, W2 = st.L[5].x, W3 = st.L[5].y, W4 = st.L[6].x,
                 W5 = st.L[6].y;
    // ---- stage 1: V_r = sum_m P_{rm} w_m (p_r first on lane s).  The six start values V = S m_s
    // only READ the DPP sources S, and put any earlier VALU write of S two instructions back
    double V0, V1, V2, V3, V4, V5;
    asm volatile(
        "v_mul_f64 %0, %6, %18\n\t"
        "v_mul_f64 %1, %7, %18\n\t"
        "v_mul_f64 %2, %8, %18\n\t"
        "v_mul_f64 %3, %9, %18\n\t"
        "v_mul_f64 %4, %10, %18\n\t"
        "v_mul_f64 %5, %11, %18\n\t"
        "v_fmac_f64_dpp %0, %6, %12 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %6, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %6, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %6, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %6, %12 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %6, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %6, %13 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %7, %13 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %7, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %7, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %7, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %7, %13 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %6, %14 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %7, %14 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %14 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %8, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %8, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %6, %15 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %7, %15 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %15 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %9, %15 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %9, %15 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %9, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %6, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %7, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %9, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %10, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %10, %16 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %6, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %7, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %9, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %10, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %11, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf"
        : "=&v"(V0), "=&v"(V1), "=&v"(V2), "=&v"(V3), "=&v"(V4), "=&v"(V5)
        : "v"(S0), "v"(S1), "v"(S2), "v"(S3), "v"(S4), "v"(S5), "v"(W0), "v"(W1), "v"(W2), "v"(W3), "v"(W4),
          "v"(W5), "v"(m_s));
    // ---- stage 2: x rows (A's columns x0, x1: their one entry), then the u rows on the s and u
    // lanes (bank 2) and the A^T (P B) sums on the x lanes (banks 0-1) into the same accumulators.
    // The s_nop covers a register copy of a W the compiler might place just before the block.
    double Q0 = H0, Q1 = H1, Q2 = H2, Q3 = H3, Q4 = H4, Q5 = H5, U0 = st.L[3].x, U1 = st.L[3].y;
    asm volatile(
        "s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %14, %8 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %15, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %14, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %14, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %14, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %14, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %14, %8 row_newbcast:9 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %7, %14, %8 row_newbcast:10 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %2, %15, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %15, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %15, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %15, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %15, %9 row_newbcast:9 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %7, %15, %9 row_newbcast:10 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %2, %16, %10 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %16, %10 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %16, %10 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %16, %10 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %16, %10 row_newbcast:9 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %7, %16, %10 row_newbcast:10 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %2, %17, %11 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %17, %11 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %17, %11 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %17, %11 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %17, %11 row_newbcast:9 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %7, %17, %11 row_newbcast:10 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %2, %18, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %18, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %18, %12 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %18, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %18, %12 row_newbcast:9 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %7, %18, %12 row_newbcast:10 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %2, %19, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %19, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %19, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %19, %13 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %19, %13 row_newbcast:9 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %7, %19, %13 row_newbcast:10 row_mask:0xf bank_mask:0x4\n\t"
        "v_fmac_f64_dpp %6, %8, %14 row_newbcast:9 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %7, %8, %14 row_newbcast:10 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %6, %9, %15 row_newbcast:9 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %7, %9, %15 row_newbcast:10 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %6, %10, %16 row_newbcast:9 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %7, %10, %16 row_newbcast:10 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %6, %11, %17 row_newbcast:9 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %7, %11, %17 row_newbcast:10 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %6, %12, %18 row_newbcast:9 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %7, %12, %18 row_newbcast:10 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %6, %13, %19 row_newbcast:9 row_mask:0xf bank_mask:0x3\n\t"
        "v_fmac_f64_dpp %7, %13, %19 row_newbcast:10 row_mask:0xf bank_mask:0x3"
        : "+v"(Q0), "+v"(Q1), "+v"(Q2), "+v"(Q3), "+v"(Q4), "+v"(Q5), "+v"(U0), "+v"(U1)
        : "v"(V0), "v"(V1), "v"(V2), "v"(V3), "v"(V4), "v"(V5), "v"(W0), "v"(W1), "v"(W2), "v"(W3), "v"(W4),
          "v"(W5));
    // the stage data are consumed: the previous step's value function goes out, the next step's
    // record (slot j - 1 - lo; at j = lo a harmless re-read) loads behind the factor and update
    __builtin_amdgcn_sched_barrier(0);
    store(po);
    nx = load(j > lo ? j - 1 - lo : 0);
    __builtin_amdgcn_sched_barrier(0);
    // ---- factor: Huu' = [[a, b], [b, d]] (a on lane u0, b and d on lane u1), every lane
    const double fa = rowchain::bcast<kLU0>(U0), fb = rowchain::bcast<kLU1>(U0), fd = rowchain::bcast<kLU1>(U1);
    const double det = fma(fa, fd, -fb * fb);
    const double r0 = rcp64(fa), rdet = rcp64(det);
    const double t = fb * r0;
    const double r1 = fa * rdet;
    // ---- update: P_k(i, c) = Hxx'(i, c) - (r0 h0_i) h0_c - (r1 h1_i) h1_c, (r h)_i from lane x_i;
    // h0_c = U0 (lane s: gu0), h1_c = U1 - t U0.  R0 is written two VALU instructions before its
    // first DPP read, R1 six
    double R0, R1, h1c;
    asm volatile(
        "v_mul_f64 %7, %9, %11\n\t"
        "v_fma_f64 %6, -%12, %11, %13\n\t"
        "v_mul_f64 %8, %10, %6\n\t"
        "v_fmac_f64_dpp %0, -%7, %11 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%7, %11 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, -%7, %11 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, -%7, %11 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, -%7, %11 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, -%7, %11 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, -%8, %6 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%8, %6 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, -%8, %6 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, -%8, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, -%8, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, -%8, %6 row_newbcast:5 row_mask:0xf bank_mask:0xf"
        : "+v"(Q0), "+v"(Q1), "+v"(Q2), "+v"(Q3), "+v"(Q4), "+v"(Q5), "=&v"(h1c), "=&v"(R0), "=&v"(R1)
        : "v"(r0), "v"(r1), "v"(U0), "v"(t), "v"(U1));
    S0 = Q0, S1 = Q1, S2 = Q2, S3 = Q3, S4 = Q4, S5 = Q5;
    no = Out{op + (long)j * ostride, {S0, S1, S2, S3, S4, S5}};
    // fac_ok of this step (riccati.h): pivots 1/d0 and d0/det positive and finite
    const bool okj = r0 > 0.0 && r0 < INFINITY && r1 > 0.0 && r1 < INFINITY;
    return !__builtin_amdgcn_readfirstlane((int)okj);
  };
  Stage sa = load(hi - lo), sb;
  for (;;) {
    int j = hi;
    for (; j > lo; j -= 2) {
      if (step(j, sa, sb, oa, ob)) return true;
      if (step(j - 1, sb, sa, ob, oa)) return true;
    }
    if (j == lo) {
      if (step(lo, sa, sb, oa, ob)) return true;
      oa = ob;
    }
    if (lo == 0) break;
    hi = lo - 1;
    lo = hi >= kWin ? hi - kWin + 1 : 0;
    // the window's reads were issued before these writes, and a wave's LDS operations complete in
    // order: the node lanes refill the ring without a wait
    asm volatile("" ::: "memory");
    fill(lo, hi, false);
    asm volatile("" ::: "memory");
    sa = load(hi - lo);
  }
  store(oa);  // node 0's
  return false;
}

}  // namespace rowchain6

}  // namespace mpcx
