// mfma_chain.h -- the backward Riccati recursion of a one-instance wave as a chain of FP64 matrix
// (MFMA) steps (gfx950 device code; DESIGN.md §3.1 "The Riccati chain on the matrix cores").
//
// The sequential chain of riccati.h runs one step per node on ONE lane while the wave issues it
// for all 64 (≈130 VALU instructions per unicycle step).  Here the whole wave runs each step as a
// few 4x4x4 FP64 MFMAs (v_mfma_f64_4x4x4_4b_f64: four independent 4x4x4 products side by side;
// all four blocks compute the same product, so each holds every result and the products chain
// without lane moves).  The step works on the AUGMENTED state z = (x, 1) (NX + 1 = 4 for the
// unicycle): the value function V(x) = 1/2 x'Px + p'x + const is the symmetric 4x4
//   S = [[P, p], [p', s]],
// the stage's dynamics dx+ = A dx + B du + c are  z+ = Gz z + Gu u  with
//   Gz = [[A, c], [0, 1]],  Gu = [[B], [0]],
// and the stage Hessian + Sigma + delta with the barrier gradient gp is the augmented
//   H = [[Hxx, gx, Hxu], [gx', 0, gu'], [Hux, gu, Huu]].
// One step (the Schur complement of the u block of G'S'G + H, G = [Gz Gu]):
//   XZ = S' Gz,  XU = S' Gu                          (MFMA 1a, 1b)
//   Mzz = Gz' XZ + Hzz,  Muz = Gu' XZ + Huz,  Muu = Gu' XU + Huu     (MFMA 2a-c)
//   Yu = -adj(Muu) Muz,  T = Muz' Yu                (MFMA 3; 2x2 adjugate from three broadcast entries)
//   S = Mzz + T / det(Muu),  Y = Yu / det(Muu)       (Y = [K | kf], the gains)
// (carried with a scale factor that keeps the exact division off the chain: mfma_chain below)
// S[x][x] = P_k, S[x][1] = p_k and Y = [K_k | kf_k]: the quantities riccati_step + riccati_gains
// give, as one homogeneous recursion (rounding differs: products are summed in the MFMA's order).
//
// Operand layouts (v_mfma_f64_4x4x4_4b_f64; measured by tools/mfma_f64_probe.hip,
// profiles/r04_mfma_probe.json): block b = (lane >> 2) & 3 is one 4x4x4 product, and with
// r = lane >> 4 (the wave's 16-lane row) and c = lane & 3: A[i][k] at (r = k, c = i), B[k][j] at
// (r = k, c = j), C/D[i][j] at (r = i, c = j).  So a D register is the B operand of the next
// product as it stands and the A operand of its TRANSPOSE (S is symmetric; Muz' = Mzu), and the
// registers that hold Gz / Gu as B operands hold Gz' / Gu' as A operands.  Every block reads the
// same entries, so all four compute the same product.
//
// Data flow: before the chain every node's lane writes its stage into a per-node LDS record
// (mc_write_record, node-parallel); during the chain each lane reads, per step, the one entry of
// each operand its position needs (five ds_read_b64, independent of the chain: issued ahead);
// each step's S and Y go to a per-node LDS output record, which every node's lane reads back after
// the chain (mc_read_result).  Used by the unicycle kernels whose wave holds one instance
// (kernels.h kMfma); NX = 3, NU = 2.
#pragma once
#include <hip/hip_runtime.h>

#include "collectives.h"
#include "riccati.h"

namespace mpcx {

constexpr int kMcMaxN = 31;  // horizons the LDS records are sized for (longer: the VALU chain)
constexpr int kMcIn = 40;    // input record: A 9, c 3, B 6, Hd 15 (packed over z = (x, u)), gp 5, 0, 1
constexpr int kMcOut = 32;   // output record: S (4x4, at 4i + j), Y (rows u, cols z, at 16 + 4u + j)
constexpr int kMcA = 0, kMcC = 9, kMcB = 12, kMcH = 18, kMcG = 33, kMcZero = 38, kMcOne = 39;
constexpr int kMcLdsDoubles = (kMcMaxN + 1) * kMcIn + kMcMaxN * kMcOut;

// record of node k: A_k (zero at node 0: interval 0 integrates from the parameter x0), c_k, B_k,
// the stage Hessian + Sigma + delta (packed, NZ = 5) and the barrier gradient
__device__ __forceinline__ void mc_write_record(double* rec, const double* Hd, const double* gp, const double* A,
                                                const double* Bm, const double* c, bool a_zero) {
#pragma unroll
  for (int i = 0; i < 9; ++i) rec[kMcA + i] = a_zero ? 0.0 : A[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) rec[kMcC + i] = c[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) rec[kMcB + i] = Bm[i];
#pragma unroll
  for (int i = 0; i < 15; ++i) rec[kMcH + i] = Hd[i];
#pragma unroll
  for (int i = 0; i < 5; ++i) rec[kMcG + i] = gp[i];
  rec[kMcZero] = 0.0;
  rec[kMcOne] = 1.0;
}

// which record entry each lane reads for each operand: position (r, q) = (lane >> 4, lane & 3)
struct McIdx {
  int gz, gu, hzz, huz, huu;
};
__device__ __forceinline__ McIdx mc_index(int lane) {
  const int r = lane >> 4, q = lane & 3;  // B / D layout: (row r, column q)
  McIdx x;
  // Gz[r][q] (B operand, k = r): A[r][q], c[r] in column 3, (0 0 0 1) in row 3
  x.gz = r < 3 ? (q < 3 ? kMcA + 3 * r + q : kMcC + r) : (q < 3 ? kMcZero : kMcOne);
  // Gu[r][q]: B[r][q] for r < 3, q < 2
  x.gu = (r < 3 && q < 2) ? kMcB + 2 * r + q : kMcZero;
  // Hzz[r][q] (D layout): Hxx, gx in row / column 3, 0 at (3, 3)
  x.hzz = (r < 3 && q < 3) ? kMcH + symix(r, q, 5) : (r < 3) ? kMcG + r : (q < 3) ? kMcG + q : kMcZero;
  // Huz[r][q]: Hux (u row r < 2), gu in column 3
  x.huz = r < 2 ? (q < 3 ? kMcH + symix(3 + r, q, 5) : kMcG + 3 + r) : kMcZero;
  // Huu[r][q]
  x.huu = (r < 2 && q < 2) ? kMcH + symix(3 + r, 3 + q, 5) : kMcZero;
  return x;
}

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// value of lane `src` (wave-uniform) through two v_readlane_b32
__device__ __forceinline__ double mc_readlane(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The chain, steps N-1 .. 0, run by every lane of the wave (one instance per wave).  rin / rout:
// the wave's input / output records in LDS.  Returns the inertia verdict: every step's Huu'
// positive definite (its LDL^T pivots a and det / a positive and finite, riccati.h fac_ok).
//
// Latency, not issue, bounds the chain (one wave per SIMD: a dependent FP64 VALU operation ≈ 30
// cycles, a dependent 4x4x4 FP64 MFMA 52-68, profiles/r04_mfma_probe.json), so the step keeps
// the exact reciprocal of det(Muu) off its critical path: the chain carries St = sig S for a
// wave-uniform scale sig, and divides by det only approximately (v_rcp_f64, relative error
// <= 4.6e-8), folding the error into the next scale:
//   Mt = G' St G + sig H = sig M,   dt = det(Mt_uu) = sig^2 det,   rho = v_rcp_f64(dt)
//   St+ = rho (dt Mt_zz - Mt_zu adj(Mt_uu) Mt_uz) = (rho dt) sig S+,   sig+ = sig (rho dt)
// so the chain's path is two products, the three entries of Mt_uu, dt (2 operations), rho (1) and
// St+ (1).  The exact results -- S+ = St+ / sig+ and Y = -adj(Mt_uu) Mt_uz / dt (sig cancels) --
// are formed beside it with full-precision reciprocals and written to the output record.
__device__ __forceinline__ bool mfma_chain(const double* rin, double* rout, int N) {
  int lane = (int)(threadIdx.x & 63);
  asm volatile("" : "+v"(lane));  // the per-lane indices are formed here, not hoisted kernel-wide
  const int r = lane >> 4;
  const McIdx ix = mc_index(lane);
  double St = rin[N * kMcIn + ix.hzz];  // terminal: [[Sigma_x + delta, gp_x], [gp_x', 0]], sig = 1
  double sig = 1.0;
  bool ok = true;
  // operands of step s (one LDS entry per operand and lane; independent of the chain)
  double gz = rin[(N - 1) * kMcIn + ix.gz], gu = rin[(N - 1) * kMcIn + ix.gu];
  double hzz = rin[(N - 1) * kMcIn + ix.hzz], huz = rin[(N - 1) * kMcIn + ix.huz], huu = rin[(N - 1) * kMcIn + ix.huu];
  const bool r0 = (r & 1) == 0;
  const bool yb = (lane & 4) != 0;  // block 1 writes Y, block 0 S (blocks 2, 3 the same again)
  double* wr = rout + (yb ? 16 : 0) + 4 * r + (lane & 3);
  for (int s = N - 1; s >= 0; --s) {
    const double XZ = mfma4(St, gz, 0.0), XU = mfma4(St, gu, 0.0);
    const double Muu = mfma4(gu, XU, sig * huu);
    const double Muz = mfma4(gu, XZ, sig * huz);
    const double Mzz = mfma4(gz, XZ, sig * hzz);
    if (s > 0) {  // next step's operands, loaded under this step's products
      const double* q = rin + (s - 1) * kMcIn;
      gz = q[ix.gz];
      gu = q[ix.gu];
      hzz = q[ix.hzz];
      huz = q[ix.huz];
      huu = q[ix.huu];
    }
    // the three entries of Mt_uu (lanes 0, 1 and 17), wave-uniform; Yu = -adj(Mt_uu) Mt_uz from
    // rows 0 and 1 of Mt_uz on both rows of each row pair (v_permlane16_swap; rows 2 and 3 pair
    // the zero rows 2, 3)
    const double a = mc_readlane(Muu, 0), b = mc_readlane(Muu, 1), d = mc_readlane(Muu, 17);
    const Pair m01 = rows16(Muz);
    const double Yu = fma(r0 ? -d : b, m01.a, (r0 ? b : -a) * m01.b);
    const double T = mfma4(Muz, Yu, 0.0);  // Mt_uz' Yu = -Mt_zu adj(Mt_uu) Mt_uz
    const double dt = fma(a, d, -b * b);
    const double rho = __builtin_amdgcn_rcp(dt);
    St = rho * fma(dt, Mzz, T);
    const double sn = sig * (rho * dt);
    // exact results beside the chain
    const double rdt = rcp64(dt);
    ok = ok && a > 0.0 && dt > 0.0 && a * rdt < INFINITY;  // LDL^T pivots a, det / a (fac_ok)
    wr[s * kMcOut] = yb ? Yu * rdt : St * rcp64(sn);
    sig = sn;
  }
  return ok;
}

// node k's results (k < N): the value function P_k (packed), p_k, and the gains K_k (NU x NX), kf_k
__device__ __forceinline__ void mc_read_value(const double* rout, int k, double* P, double* p) {
  const double* o = rout + k * kMcOut;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = i; j < 3; ++j) P[symix(i, j, 3)] = o[4 * i + j];
    p[i] = o[4 * i + 3];
  }
}
__device__ __forceinline__ void mc_read_gains(const double* rout, int k, double* K, double* kf) {
  const double* o = rout + k * kMcOut;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
#pragma unroll
    for (int j = 0; j < 3; ++j) K[u * 3 + j] = o[16 + 4 * u + j];
    kf[u] = o[16 + 4 * u + 3];
  }
}

}  // namespace mpcx
