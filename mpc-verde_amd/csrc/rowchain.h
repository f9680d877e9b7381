// rowchain.h -- the unicycle's backward Riccati recursion with every step spread over a 16-lane row
// (gfx950 device code; DESIGN.md §3.1 "row chain").
//
// The sequential recursion of riccati.h runs step j on node lane j alone: ~110 FP64 operations
// issued for the whole wave to use one lane, plus 18 DPP moves of (P, p) to the next lane.  Here
// the same step -- the same operations in the same order, so the same bits -- is computed by the
// lanes of a 16-lane row, each lane owning one COLUMN of the step's products:
//
//   row lane   0   1   2   4   5   6        (3, 7..15: a dummy column, never read)
//   column     x0  x1  x2  s   u0  u1       s = the value function's affine part (P c + p, g)
//
// (the x lanes in DPP bank 0, the s and u lanes in bank 1: the u-row sums of the s and u lanes and
// the x lanes' A^T (P B) sums accumulate into the same registers through bank-masked FMAs)
// and every operand another lane owns arrives as the DPP row_newbcast source of a v_fmac_f64
// (gfx950's 64-bit DPP: lane E of the row broadcast to the row inside the FMA, no separate move).
// The value function stays where the step leaves it: lane c holds column c of P_k (rows i <= c
// are the upper triangle the recursion keeps) and lane s holds p_k, so P_{nm} of the next step is
// the broadcast of lane max(n, m), register min(n, m).  A step is
//   stage 1  V_{.b} = P W_b (+ p on lane s): W_b = column b of [A c B], lane-held (9 FMAs)
//   stage 2  Q_{ab} = H_{ab} + sum_m W_{ma} V_{mb}: W_{ma} broadcast from lane a (Hxx', Huu', gx, gu)
//   h-seq    Hux' = H + A^T (P B) on the x lanes, from lanes u0/u1's V (the A^T (P B) order of
//            riccati.h kAtPB, which the column lanes cannot take from stage 2 themselves), into the
//            registers that hold the u rows on the s and u lanes
//   factor   the 2x2 L D L^T of Huu' (every lane, from three broadcasts)
//   update   P_k = Hxx' - (r0 h0) h0^T - (r1 h1) h1^T, column c on lane c, (r h)_i from lane x_i
// about 60 VALU instructions instead of ~128, with every row holding an instance's whole chain:
// no row ever needs another row, so the replicated (R = 2), narrow 32-lane and 64-lane groups all
// run it unchanged.  Stage data reach the rows through LDS records that the node lanes write
// before the chain (one 8-double column block per lane: H column, then the column's W entries).
// The chain hands back only the value function: after step j the x and s lanes of the instance's
// first row store P_j's columns into node j's record, and after the chain node lane k redoes its
// own step from node k+1's value function -- riccati_step, all nodes at once -- for its factors
// and P_k (the same function on the same operands as the chain's step k, so the same bits).
// tests/hip/rowchain_check.hip compares the chain with riccati_step bit for bit.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "collectives.h"
#include "riccati.h"

namespace mpcx {

namespace rowchain {

// diagnostic switches of tools/rowchain_probe.py (timing of the chain's parts in the test harness only;
// 0 in every product build): 1 = no value-function stores, 2 = no stage loads after the first
#ifndef MPCX_ROWCHAIN_PROBE
#define MPCX_ROWCHAIN_PROBE 0
#endif

constexpr int kBlk = 8;                // doubles per column block: H_{0..4,b}, W_{0..2,b}
constexpr int kCols = 7;               // x0 x1 x2 s u0 u1 dummy
// doubles per node record: 7 blocks of 8, padded to 58 so that the node lanes' records start in
// different LDS banks (a 448-byte stride sends every fourth node lane to the same banks)
constexpr int kRec = kBlk * kCols + 2;
constexpr int kBS = 3, kBU0 = 4;        // blocks (columns) of s and u0 (x_c: block c; u1: 5)
constexpr int kLX2 = 2, kLS = 4, kLU0 = 5, kLU1 = 6;  // lanes of x2, s, u0, u1 (x_c on lane c)
// the value function P_j in node j's record (after its stage data are consumed): column c of P_j
// (x0..x2; c = s: p_j) in slots [2..4] of block c

// the model's structure the chain hard-codes (the unicycle: A = I + a02 e0 e2^T + a12 e1 e2^T,
// B[2][0] = 0; riccati.h takes Hux' as A^T (P B))
template <class Model>
constexpr bool fits() {
  return Model::NX == 3 && Model::NU == 2 &&
         Model::AMASK == ((1ull << 0) | (1ull << 2) | (1ull << 4) | (1ull << 5) | (1ull << 8)) &&
         Model::BMASK == ((1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3) | (1ull << 5)) &&
         AOneOf<Model>::value == ((1ull << 0) | (1ull << 4) | (1ull << 8)) &&
         hux_by_atpb<3, 2, Model::AMASK, Model::BMASK>();
}

// node k's stage into its record (node lane k < N, before the chain; 16-byte stores).  Block b
// holds column b of the stage's bordered Hessian [[Hd, g], [g^T, .]] and column b of [A c B] as the
// chain's stage 1 takes it: x2 without its unit entry (stage 1 starts from P's column 2 instead),
// the structural ones and zeros as constants.
__device__ __forceinline__ void store_stage(double* rk, const double* Hd, const double* gp, const double* A,
                                            const double* Bm, const double* c) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  auto put = [&](int b, int q, double x, double y) __attribute__((always_inline)) {
    *reinterpret_cast<v2d*>(rk + b * kBlk + 2 * q) = v2d{x, y};
  };
  // H columns: x0, x1, x2 (Hd columns 0..2), s (the barrier gradient), u0, u1 (Hd columns 3, 4)
  constexpr int hcol[6] = {0, 1, 2, -1, 3, 4};
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    double h[5];
#pragma unroll
    for (int a = 0; a < 5; ++a) h[a] = hcol[b] < 0 ? gp[a] : Hd[symix(a, hcol[b], 5)];
    double w[3];
    switch (b) {
      case 0: w[0] = 1.0, w[1] = 0.0, w[2] = 0.0; break;
      case 1: w[0] = 0.0, w[1] = 1.0, w[2] = 0.0; break;
      case 2: w[0] = A[2], w[1] = A[5], w[2] = 0.0; break;       // A02, A12 (A22 = 1: stage 1's start)
      case 3: w[0] = c[0], w[1] = c[1], w[2] = c[2]; break;
      case 4: w[0] = Bm[0], w[1] = Bm[2], w[2] = 0.0; break;      // B00, B10 (B20 = 0)
      default: w[0] = Bm[1], w[1] = Bm[3], w[2] = Bm[5]; break;  // B01, B11, B21
    }
    put(b, 0, h[0], h[1]);
    put(b, 1, h[2], h[3]);
    put(b, 2, h[4], w[0]);
    put(b, 3, w[1], w[2]);
  }
}

// node N's value function, the chain's starting point: P_N = diag(Sigma_x + delta), p_N = gradient;
// the u lanes and the dummy lanes start from zeros (their stage-1 start is multiplied by 0, which
// must not meet an inf or NaN from uninitialised LDS)
__device__ __forceinline__ void store_terminal(double* rk, const double* P, const double* p) {
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int i = 0; i < 3; ++i) rk[c * kBlk + 2 + i] = P[symix(i, c, 3)];
#pragma unroll
  for (int i = 0; i < 3; ++i) rk[kBS * kBlk + 2 + i] = p[i];
#pragma unroll
  for (int c = kBU0; c < kCols; ++c)
#pragma unroll
    for (int i = 0; i < 3; ++i) rk[c * kBlk + 2 + i] = 0.0;
}

// node k+1's value function after the chain (node lane k < N reads record k + 1): the operands of
// its own riccati_step, exactly as the sequential recursion hands them on (P upper triangle, p)
__device__ __forceinline__ void load_next(const double* rk1, double* P, double* p) {
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int i = 0; i <= c; ++i) P[symix(i, c, 3)] = rk1[c * kBlk + 2 + i];
#pragma unroll
  for (int i = 0; i < 3; ++i) p[i] = rk1[kBS * kBlk + 2 + i];
}

// v_mov_b64 with a DPP row_newbcast source (the compiler sees the DPP and inserts its hazard waits)
template <int E>
__device__ __forceinline__ double bcast(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + E, 0xf, 0xf, true);
}

// The chain: steps N-1 .. 0 over the records of the row's instance.  Every lane of the wave runs
// it (a broadcast source must be active); `rec` = the row's instance's node-0 record.  Each group
// of DPP FMAs is one asm statement behind one s_nop 1: the VALU-write -> DPP-read hazard of its
// sources, which the compiler does not see inside the asm, is covered once, and no source is
// written inside a group.
template <int GR>  // lanes per instance on the wave (G R <= 64)
__device__ __forceinline__ void run(const double* rec, int N) {
  // the lane constants below are derived here, inside the solve loop: opaque to loop-invariant code
  // motion, which would otherwise hoist them out of the solve loop and hold their registers across
  // every phase of it
  int r = (int)(threadIdx.x & 15);
  asm volatile("" : "+v"(r));
  const int col = r < kLX2 + 1 ? r : (r >= kLS && r <= kLU1) ? r - 1 : 6;  // block of this lane's column
  // lane constants: the stage-1 start (P's column on lane x2, p on lane s), the unit terms of A's
  // column 2 in the orders riccati.h sums them (last on the x and s lanes, first on the u lanes),
  // A22 = 1 of the h-sequence on lane x2
  const double m_x2s = (r == kLX2 || r == kLS) ? 1.0 : 0.0;
  const double m_u = (r == kLU0 || r == kLU1) ? 1.0 : 0.0;
  const double m_xs = r <= kLS ? 1.0 : 0.0;
  const double m_x2 = r == kLX2 ? 1.0 : 0.0;
  double* base = const_cast<double*>(rec) + col * kBlk;  // this lane's column block of node 0
  typedef double v2d __attribute__((ext_vector_type(2)));
  auto ld2 = [&](const double* p) __attribute__((always_inline)) { return *reinterpret_cast<const v2d*>(p); };

  // value function of node N (this lane's column)
  double S0 = base[N * kRec + 2], S1 = base[N * kRec + 3], S2 = base[N * kRec + 4];
  // a step's stage data: the block's four pairs
  struct Stage {
    v2d L0, L1, L2, L3;
  };
  auto load = [&](int j) __attribute__((always_inline)) {
    const double* rn = base + j * kRec;
    return Stage{ld2(rn + 0), ld2(rn + 2), ld2(rn + 4), ld2(rn + 6)};
  };
  // a step's results (into its own record, one step later)
  struct Out {
    double* r;
    double s0, s1, s2;
  };
  // only the x and s lanes of an instance's first row store (the other rows hold the same bits):
  // rows writing the same addresses would serialise in LDS.  One asm statement under those lanes'
  // exec mask -- no branch around it (an exec-masked `if` costs a basic block and its branch every
  // step).  The compiler does not see these LDS writes: the reads of them come later from the same
  // wave, and a wave's LDS operations complete in order, so no wait is needed for them.
  int lw = (int)(threadIdx.x & 63) % GR;
  asm volatile("" : "+v"(lw));
  const unsigned long long wmask = __ballot((r <= kLX2 || r == kLS) && lw < 16);
  auto store = [&](const Out& o) __attribute__((always_inline)) {
    const unsigned a = (unsigned)(unsigned long)((__attribute__((address_space(3))) double*)o.r);
    unsigned long long saved;
    asm volatile(
        "s_and_saveexec_b64 %0, %1\n\t"
        "ds_write2_b64 %2, %3, %4 offset0:2 offset1:3\n\t"
        "ds_write_b64 %2, %5 offset:32\n\t"
        "s_or_b64 exec, exec, %0"
        : "=&s"(saved)
        : "s"(wmask), "v"(a), "v"(o.s0), "v"(o.s1), "v"(o.s2)
        : "memory", "scc");  // (the exec save / restore sets SCC)
  };
  // one step on the loaded stage `st`, issuing the loads of the next step (record j - 1; at j = 0 a
  // harmless re-read of record 0) into `nx` after stage 2, so their latency hides behind the step;
  // the previous step's results `po` go out, this step's are `no`.  Two stage and two result
  // variables alternate between consecutive steps (the loop below is unrolled by two): a single
  // loop-carried set would cost register copies at every back edge
  auto step = [&](auto prev, int j, const Stage& st, Stage& nx, const Out& po, Out& no) __attribute__((always_inline)) {
    double* rj = base + j * kRec;
    const double H0 = st.L0.x, H1 = st.L0.y, H2 = st.L1.x, H3 = st.L1.y, H4 = st.L2.x;
    const double cf0 = st.L2.y, cf1 = st.L3.x, cf2 = st.L3.y;
    // ---- stage 1: V_m = P(m, .) W_b, P(m, 2) first on lane x2 and p_m first on lane s.  The start
    // values V = S * m (three VALU writes that only READ the DPP sources S) open the block, so any
    // earlier VALU write of S is at least two wait states before the first DPP read: no s_nop
    double V0, V1, V2;
    asm volatile(
        "v_mul_f64 %0, %3, %9\n\t"
        "v_mul_f64 %1, %4, %9\n\t"
        "v_mul_f64 %2, %5, %9\n\t"
        "v_fmac_f64_dpp %0, %3, %6 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"  // V0 += P00 w0
        "v_fmac_f64_dpp %1, %3, %6 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"  // V1 += P10 w0
        "v_fmac_f64_dpp %2, %3, %6 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"  // V2 += P20 w0
        "v_fmac_f64_dpp %0, %3, %7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"  // V0 += P01 w1
        "v_fmac_f64_dpp %1, %4, %7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"  // V1 += P11 w1
        "v_fmac_f64_dpp %2, %4, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"  // V2 += P21 w1
        "v_fmac_f64_dpp %0, %3, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"  // V0 += P02 w2
        "v_fmac_f64_dpp %1, %4, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"  // V1 += P12 w2
        "v_fmac_f64_dpp %2, %5, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf"      // V2 += P22 w2
        : "=&v"(V0), "=&v"(V1), "=&v"(V2)
        : "v"(S0), "v"(S1), "v"(S2), "v"(cf0), "v"(cf1), "v"(cf2), "v"(m_x2s));
    // the stage data are being consumed; the next step's record (j - 1; at j = 0 a harmless re-read of
    // record 0) loads into the other register set while this step runs, and the previous step's
    // results go out first (LDS operations complete in order, so the next step's wait covers them)
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (decltype(prev)::value)
      if (!(MPCX_ROWCHAIN_PROBE & 1)) store(po);
    if (!(MPCX_ROWCHAIN_PROBE & 2)) nx = load(j > 0 ? j - 1 : 0);
    else nx = st;
    __builtin_amdgcn_sched_barrier(0);
    // ---- stage 2 and the factor in one block, so that the x rows fill the reciprocals' latency.
    // Stage 2: Q_a = H_a + sum_m W_{m a} V_m (a = x0, x1, x2, u0, u1), W_{m a} from lane a -- the u
    // rows on the s and u lanes (bank 1) -- and the h-sequence on the x lanes (bank 0), into the same
    // registers: Hux'(l, c) = H(u_l, x_c) + (A^T (P B))(c, l) on lane x_c, (P B) from lane u_l
    // (riccati.h kAtPB's order, which the column lanes cannot take from stage 2).  Factor: Huu' =
    // [[a, b], [b, d]] (a on lane u0, b and d on lane u1) on every lane, det = a d - b^2, r0 = 1/a and
    // 1/det as rcp64 (v_rcp_f64 and two Newton steps), t = b r0, r1 = a / det -- riccati.h's operations
    // in its order.  The DPP sources are LDS loads, V (stage 1, at least ten instructions back) and Q3 /
    // Q4 (last written three and four instructions before their broadcasts)
    double Q0, Q1, Q2, Q3 = H3, Q4 = H4, r0, t, r1, fa, fb, fd, det, rdet, e0, e1;
    asm volatile(
        "v_fmac_f64_dpp %3, %21, %18 row_newbcast:5 row_mask:0xf bank_mask:0x2\n\t"  // Q3 + B00 V0
        "v_fmac_f64_dpp %4, %21, %18 row_newbcast:6 row_mask:0xf bank_mask:0x2\n\t"  // Q4 + B01 V0
        "v_fmac_f64_dpp %3, %22, %19 row_newbcast:5 row_mask:0xf bank_mask:0x2\n\t"  // + B10 V1
        "v_fmac_f64_dpp %4, %22, %19 row_newbcast:6 row_mask:0xf bank_mask:0x2\n\t"  // + B11 V1
        "v_fmac_f64_dpp %4, %23, %20 row_newbcast:6 row_mask:0xf bank_mask:0x2\n\t"  // + B21 V2
        "v_fmac_f64_dpp %3, %20, %26 row_newbcast:5 row_mask:0xf bank_mask:0x1\n\t"  // + (PB)_20 [A22 on x2]
        "v_fmac_f64_dpp %4, %20, %26 row_newbcast:6 row_mask:0xf bank_mask:0x1\n\t"
        "v_fmac_f64_dpp %3, %18, %21 row_newbcast:5 row_mask:0xf bank_mask:0x1\n\t"  // + (PB)_00 A0c
        "v_fmac_f64_dpp %4, %18, %21 row_newbcast:6 row_mask:0xf bank_mask:0x1\n\t"
        "v_fmac_f64_dpp %3, %19, %22 row_newbcast:5 row_mask:0xf bank_mask:0x1\n\t"  // + (PB)_10 A1c
        "v_fmac_f64_dpp %4, %19, %22 row_newbcast:6 row_mask:0xf bank_mask:0x1\n\t"
        "v_add_f64 %0, %15, %18\n\t"          // Q0 = H0 + V0 (A00 = 1: column x0's only term)
        "v_add_f64 %1, %16, %19\n\t"          // Q1 = H1 + V1
        "v_mov_b64_dpp %8, %3 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"   // a
        "v_mov_b64_dpp %9, %3 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"   // b
        "v_mov_b64_dpp %10, %4 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"  // d
        "v_rcp_f64 %5, %8\n\t"                // r0 ~ 1/a
        "v_mul_f64 %11, %9, -%9\n\t"          // det = -b b
        "v_fmac_f64 %11, %8, %10\n\t"         //       + a d
        "v_fma_f64 %2, %20, %24, %17\n\t"     // Q2 = H2 + V2 on the u lanes (A22's unit term first there)
        "v_rcp_f64 %12, %11\n\t"              // rdet ~ 1/det
        "v_fma_f64 %13, -%8, %5, 1.0\n\t"
        "v_fmac_f64_dpp %2, %21, %18 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"  // + A02 V0
        "v_fmac_f64 %5, %5, %13\n\t"
        "v_fma_f64 %14, -%11, %12, 1.0\n\t"
        "v_fmac_f64_dpp %2, %22, %19 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"  // + A12 V1
        "v_fma_f64 %13, -%8, %5, 1.0\n\t"
        "v_fmac_f64 %12, %12, %14\n\t"
        "v_fma_f64 %2, %20, %25, %2\n\t"      // + A22 V2 last on the x and s lanes
        "v_fmac_f64 %5, %5, %13\n\t"          // r0
        "v_fma_f64 %14, -%11, %12, 1.0\n\t"
        "v_mul_f64 %6, %9, %5\n\t"            // t = b r0
        "v_fmac_f64 %12, %12, %14\n\t"        // rdet
        "v_mul_f64 %7, %8, %12"               // r1 = a rdet
        : "=&v"(Q0), "=&v"(Q1), "=&v"(Q2), "+v"(Q3), "+v"(Q4), "=&v"(r0), "=&v"(t), "=&v"(r1), "=&v"(fa),
          "=&v"(fb), "=&v"(fd), "=&v"(det), "=&v"(rdet), "=&v"(e0), "=&v"(e1)
        : "v"(H0), "v"(H1), "v"(H2), "v"(V0), "v"(V1), "v"(V2), "v"(cf0), "v"(cf1), "v"(cf2), "v"(m_u),
          "v"(m_xs), "v"(m_x2));
    // lane x_c: Hux'(0, c), Hux'(1, c); lane s: gu0 (g0) and gu1 for g1 (stage 2's u rows there)
    const double h0c = Q3, hu1c = Q4;
    // ---- update: P_k(i, c) = Hxx'(i, c) - (r0 h0_i) h0_c - (r1 h1_i) h1_c, (r h)_i from lane x_i.
    // R0 is written two VALU instructions before its first DPP read, R1 three: no s_nop
    double R0, R1, h1c;
    S0 = Q0;
    S1 = Q1;
    S2 = Q2;
    asm volatile(
        "v_mul_f64 %4, %6, %8\n\t"         // R0 = r0 h0c
        "v_fma_f64 %3, -%9, %8, %10\n\t"   // h1c = hu1c - t h0c
        "v_mul_f64 %5, %7, %3\n\t"         // R1 = r1 h1c
        "v_fmac_f64_dpp %0, -%4, %8 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%4, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, -%4, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, -%5, %3 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%5, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, -%5, %3 row_newbcast:2 row_mask:0xf bank_mask:0xf"
        : "+v"(S0), "+v"(S1), "+v"(S2), "=&v"(h1c), "=&v"(R0), "=&v"(R1)
        : "v"(r0), "v"(r1), "v"(h0c), "v"(t), "v"(hu1c));
    // ---- node j's results, stored during the next step (every lane writes its own block; only the
    // columns read back matter)
    no = Out{rj, S0, S1, S2};  // stored during the next step
  };
  Stage sa = load(N - 1), sb;
  Out oa{}, ob{};
  step(std::false_type{}, N - 1, sa, sb, oa, ob);
  int j = N - 2;
  for (; j >= 1; j -= 2) {
    step(std::true_type{}, j, sb, sa, ob, oa);
    step(std::true_type{}, j - 1, sa, sb, oa, ob);
  }
  if (j == 0) step(std::true_type{}, 0, sb, sa, ob, oa);
  if (!(MPCX_ROWCHAIN_PROBE & 1)) store(j == 0 ? oa : ob);  // step 0's results
}

}  // namespace rowchain

}  // namespace mpcx
