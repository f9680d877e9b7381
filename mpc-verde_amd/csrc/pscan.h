// pscan.h -- parallel-in-time (log-depth) Riccati recursion for the fused solve kernel.
//
// The backward Riccati recursion of the barrier KKT system (riccati.h) is a chain of N
// dependent steps, executed by one lane at a time while the rest of the wave idles: at
// N = 100 (config 5) it is ~80 % of an IPM iteration.  The value functions can instead be
// computed by an associative scan over per-stage "conditional value function" elements
// (Saerkkae & Garcia-Fernandez, "Temporal parallelization of dynamic programming and linear
// quadratic control", IEEE TAC 2023): element k describes going from x_k to x_{k+1},
//
//   x_{k+1} = A_k x_k + b_k + w,   cost  1/2 x^T J_k x + p_k^T x + 1/2 w^T C_k^+ w,
//
// built by eliminating u from the stage (Q, S, R, q, r; dynamics F, L, c):
//   A = F - L R^-1 S^T,  b = c - L R^-1 r,  C = L R^-1 L^T,  J = Q - S R^-1 S^T,  p = q - S R^-1 r,
// the terminal node is (0, 0, 0, P_N, p_N), and lanes past N hold the identity (I, 0, 0, 0, 0).
// Two elements combine (e1 = i->j, e2 = j->k) as
//   M  = I + C1 J2,  T1 = A2 M^-1,  T2 = M^-1 A1
//   A  = T1 A1,      b = T1 (b1 - C1 p2) + b2,     C = T1 C1 A2^T + C2,
//   p  = T2^T (p2 + J2 b1) + p1,                   J = T2^T J2 A1 + J1,
// and the suffix e_k (x) ... (x) e_N has A = b = C = 0 and (J, p) = the value function (P_k, p_k)
// of the sequential recursion.  Lanes run a Hillis-Steele suffix scan (lane k combines with lane
// k + d, d = 1, 2, 4, ...): ceil(log2(N+1)) levels of O(NX^3) work on all lanes instead of N
// dependent steps.  The stage gains, the inertia test and the (P_k, p_k) used downstream then
// come from ONE node-parallel riccati_step per lane on P_{k+1} from the scan, and that step's
// P_k is compared with the scan's own: the caller falls back to the sequential recursion when
// a stage R is not positive definite, a value is not finite, or the two disagree
// (the combination inverts I + C1 J2 without pivoting; with C, J positive semidefinite it is
// similar to an SPD matrix, and the consistency check catches the rest).
#pragma once
#include <hip/hip_runtime.h>

#include "collectives.h"
#include "riccati.h"

namespace mpcx {

template <int NX>
struct RElem {
  static constexpr int NP = NX * (NX + 1) / 2;
  static constexpr int NE = NX * NX + 2 * NX + 2 * NP;  // doubles per element
  // field offsets (element f of lane t lives at buf[f * stride + t] in LDS)
  static constexpr int oA = 0, ob = NX * NX, oC = ob + NX, oJ = oC + NP, op = oJ + NP;
  double A[NX * NX], b[NX], C[NP], J[NP], p[NX];
};

// store lane t's element in the LDS scan buffer (structure of arrays: conflict-free)
template <int NX>
__device__ __forceinline__ void relem_store(const RElem<NX>& e, double* buf, int stride, int t) {
  using E = RElem<NX>;
#pragma unroll
  for (int i = 0; i < NX * NX; ++i) buf[(E::oA + i) * stride + t] = e.A[i];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    buf[(E::ob + i) * stride + t] = e.b[i];
    buf[(E::op + i) * stride + t] = e.p[i];
  }
#pragma unroll
  for (int i = 0; i < E::NP; ++i) {
    buf[(E::oC + i) * stride + t] = e.C[i];
    buf[(E::oJ + i) * stride + t] = e.J[i];
  }
}

// identity element (lanes past node N)
template <int NX>
__device__ __forceinline__ void relem_identity(RElem<NX>& e) {
#pragma unroll
  for (int i = 0; i < NX * NX; ++i) e.A[i] = (i % (NX + 1) == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int i = 0; i < NX; ++i) e.b[i] = e.p[i] = 0.0;
#pragma unroll
  for (int i = 0; i < RElem<NX>::NP; ++i) e.C[i] = e.J[i] = 0.0;
}

// element of stage k from the stage blocks (Hd = stage Hessian + Sigma + delta, packed over
// z = (x, u); gp = barrier gradient; A, Bm, c = dynamics).  Returns false when R = Hd_uu is
// not positive definite (the scan is then not used).
template <int NX, int NU, unsigned long long AMASK, unsigned long long BMASK>
__device__ __forceinline__ bool relem_stage(const double* Hd, const double* gp, const double* A, const double* Bm,
                                            const double* c, RElem<NX>& e) {
  constexpr int NZ = NX + NU;
  static_assert(NU == 1 || NU == 2, "NU must be 1 or 2");
  double Ri[NU * NU];
  bool ok;
  if constexpr (NU == 1) {
    const double r = Hd[symix(NX, NX, NZ)];
    ok = r > 0.0;
    Ri[0] = rcp64(r);
  } else {
    const double a = Hd[symix(NX, NX, NZ)], bb = Hd[symix(NX, NX + 1, NZ)], d = Hd[symix(NX + 1, NX + 1, NZ)];
    const double det = fma(a, d, -bb * bb);
    ok = a > 0.0 && det > 0.0;
    const double rd = rcp64(det);
    Ri[0] = d * rd;
    Ri[1] = Ri[2] = -bb * rd;
    Ri[3] = a * rd;
  }
  // LRi = L R^-1 (NX x NU), SRi = S R^-1 (NX x NU), S[i][l] = Hd(x_i, u_l)
  double LRi[NX * NU], SRi[NX * NU];
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int l = 0; l < NU; ++l) {
      double al = 0.0, as = 0.0;
#pragma unroll
      for (int m = 0; m < NU; ++m) {
        if (BMASK & (1ull << (i * NU + m))) al = fma(Bm[i * NU + m], Ri[m * NU + l], al);
        as = fma(Hd[symix(i, NX + m, NZ)], Ri[m * NU + l], as);
      }
      LRi[i * NU + l] = al;
      SRi[i * NU + l] = as;
    }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double acc = (AMASK & (1ull << (i * NX + j))) ? A[i * NX + j] : 0.0;
#pragma unroll
      for (int l = 0; l < NU; ++l) acc = fma(-LRi[i * NU + l], Hd[symix(j, NX + l, NZ)], acc);
      e.A[i * NX + j] = acc;
    }
    double bacc = c[i], pacc = gp[i];
#pragma unroll
    for (int l = 0; l < NU; ++l) {
      bacc = fma(-LRi[i * NU + l], gp[NX + l], bacc);
      pacc = fma(-SRi[i * NU + l], gp[NX + l], pacc);
    }
    e.b[i] = bacc;
    e.p[i] = pacc;
#pragma unroll
    for (int j = i; j < NX; ++j) {
      double cacc = 0.0, jacc = Hd[symix(i, j, NZ)];
#pragma unroll
      for (int l = 0; l < NU; ++l) {
        if (BMASK & (1ull << (j * NU + l))) cacc = fma(LRi[i * NU + l], Bm[j * NU + l], cacc);
        jacc = fma(-SRi[i * NU + l], Hd[symix(j, NX + l, NZ)], jacc);
      }
      e.C[symix(i, j, NX)] = cacc;
      e.J[symix(i, j, NX)] = jacc;
    }
  }
  return ok;
}

// in-place inverse of a general NX x NX matrix (Gauss-Jordan, no pivoting; see header)
template <int NX>
__device__ __forceinline__ void inv_nopiv(double* a) {
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    const double pv = rcp64(a[k * NX + k]);
    a[k * NX + k] = 1.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) a[k * NX + j] *= pv;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      if (i == k) continue;
      const double f = a[i * NX + k];
      a[i * NX + k] = 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) a[i * NX + j] = fma(-f, a[k * NX + j], a[i * NX + j]);
    }
  }
}

// e1 <- e1 (x) e2 with e2 read from the LDS scan buffer (q = buf + partner lane, fields
// `stride` apart): the partner never occupies registers, and the temporaries are ordered so
// that at most four NX x NX blocks are live besides e1
template <int NX>
__device__ __forceinline__ void relem_combine_lds(RElem<NX>& e1, const double* q, int stride) {
  using E = RElem<NX>;
  auto A2 = [&](int i, int j) { return q[(E::oA + i * NX + j) * stride]; };
  auto b2 = [&](int i) { return q[(E::ob + i) * stride]; };
  auto C2 = [&](int i, int j) { return q[(E::oC + symix(i, j, NX)) * stride]; };
  auto J2 = [&](int i, int j) { return q[(E::oJ + symix(i, j, NX)) * stride]; };
  auto p2 = [&](int i) { return q[(E::op + i) * stride]; };
  auto C1 = [&](int i, int j) { return e1.C[symix(i, j, NX)]; };
  double Mi[NX * NX];
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double acc = (i == j) ? 1.0 : 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(C1(i, m), J2(m, j), acc);
      Mi[i * NX + j] = acc;
    }
  inv_nopiv<NX>(Mi);
  {  // p, J (read the old A1, b1): T2 = Mi A1, J <- T2^T (J2 A1) + J1, p <- T2^T (p2 + J2 b1) + p1
    double T2[NX * NX], J2A1[NX * NX], v[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        double t = 0.0, u = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) {
          t = fma(Mi[i * NX + m], e1.A[m * NX + j], t);
          u = fma(J2(i, m), e1.A[m * NX + j], u);
        }
        T2[i * NX + j] = t;
        J2A1[i * NX + j] = u;
      }
      double acc = p2(i);
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(J2(i, m), e1.b[m], acc);
      v[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      double acc = e1.p[i];
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(T2[m * NX + i], v[m], acc);
      e1.p[i] = acc;
#pragma unroll
      for (int j = i; j < NX; ++j) {
        double a = e1.J[symix(i, j, NX)];
#pragma unroll
        for (int m = 0; m < NX; ++m) a = fma(T2[m * NX + i], J2A1[m * NX + j], a);
        e1.J[symix(i, j, NX)] = a;
      }
    }
  }
  // T1 = A2 Mi; b <- T1 (b1 - C1 p2) + b2, A <- T1 A1, C <- (T1 C1) A2^T + C2
  double T1[NX * NX], w[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(A2(i, m), Mi[m * NX + j], acc);
      T1[i * NX + j] = acc;
    }
    double acc = e1.b[i];
#pragma unroll
    for (int m = 0; m < NX; ++m) acc = fma(-C1(i, m), p2(m), acc);
    w[i] = acc;
  }
  double T1C1[NX * NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    double bacc = b2(i);
#pragma unroll
    for (int m = 0; m < NX; ++m) bacc = fma(T1[i * NX + m], w[m], bacc);
    e1.b[i] = bacc;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double cc = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) cc = fma(T1[i * NX + m], C1(m, j), cc);
      T1C1[i * NX + j] = cc;
    }
  }
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = i; j < NX; ++j) {
      double acc = C2(i, j);
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(T1C1[i * NX + m], A2(j, m), acc);
      e1.C[symix(i, j, NX)] = acc;
    }
  // A <- T1 A1 column by column (a column of A1 is dead once its new column is formed)
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double col[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      double a = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) a = fma(T1[i * NX + m], e1.A[m * NX + j], a);
      col[i] = a;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) e1.A[i * NX + j] = col[i];
  }
}

}  // namespace mpcx
