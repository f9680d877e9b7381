// riccati.h -- one backward step of the Riccati factorisation of the barrier KKT system,
// for a stage with NX states and NU in {1, 2} controls (gfx950 device code).
//
// The step is the sequential critical path of the fused solve, so it
// only computes what the next step needs: the value function (Pn, pn) of node k.  Huu' is
// factored as L D L^T (no square roots; the two reciprocals are independent), and the
// feedback K, k_f are recovered afterwards, on all lanes at once (riccati_gains).
// Structural zeros of A and B are compile-time masks (bit r*NX+j of AMASK = A[r][j] may
// be non-zero), so a model with sparse Jacobians gets a short step without relying on
// fast-math folding of x*0.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "collectives.h"

namespace mpcx {

// packed upper-triangular index of a symmetric n x n matrix.  Always inlined: in the largest
// kernels (the 6-state bicycle) the inliner otherwise leaves it a call, its index a run-time
// value, and every array it indexes a stack object in scratch.
__host__ __device__ constexpr __forceinline__ int symix(int i, int j, int n) {
  return i <= j ? i * n - i * (i - 1) / 2 + (j - i) : j * n - j * (j - 1) / 2 + (i - j);
}

// row i of P c for a packed symmetric P (the SREORD / DEC order)
template <int NX>
__device__ __forceinline__ double riccati_pc_row(const double* P, const double* c, int i) {
  double acc = P[symix(i, 0, NX)] * c[0];
#pragma unroll
  for (int m = 1; m < NX; ++m) acc = fma(P[symix(i, m, NX)], c[m], acc);
  return acc;
}

template <int NX, int NU>
struct Fac {  // LDL^T data of Huu' kept for the gains (per lane)
  double r0, r1, t;  // 1/d0, 1/d1, L[1][0]
  double h0[NX], h1[NX];  // rows of L^{-1} Hux'
  double g0, g1;          // L^{-1} gu'
};

//
// DEC: the stage is decoupled -- its B is zero and its stage Hessian has no x-u block -- and
// Pown holds the P_k this same step produced at the previous factorisation from identical
// operands (same stage Hessian, A and P_{k+1}; the caller guarantees it, solver.hip
// "decoupled suffix").  Then Hux' = 0, Huu' = Huu and P_k = Hxx + A^T P_{k+1} A is Pown
// itself: the step only carries the vector part, p_k = gx + A^T (p_{k+1} + P_{k+1} c),
// computed with the full step's operation order (same bits up to the sign of an exact zero).
// SREORD: s = (P_{k+1} c) + p_{k+1} with the product summed first -- the order in which the
// DEC step takes it precomputed off the chain (vpre = P_{k+1} c, riccati_pc), so the two
// variants of a model that uses DEC give the same bits.
// Model::AONE (structural unit entries of A, riccati_step) if the model declares it, else 0
template <class M, class = void>
struct AOneOf {
  static constexpr unsigned long long value = 0;
};
template <class M>
struct AOneOf<M, std::void_t<decltype(M::AONE)>> {
  static constexpr unsigned long long value = M::AONE;
};

// Model::kXBounds if the model declares it, else true: false = the model's solve kernel never
// sees finite state bounds (the launch picks it only then), so every state-bound term of the
// barrier, the complementarity, the fraction to the boundary and the bound-dual update is a
// compile-time zero
template <class M, class = void>
struct XBoundsOf {
  static constexpr bool value = true;
};
template <class M>
struct XBoundsOf<M, std::void_t<decltype(M::kXBounds)>> {
  static constexpr bool value = M::kXBounds;
};
// model trait: the stage Hessian and Sigma wait in the restoration workspace across the
// inertia-correction loop (kernels.h kWsStash; solver.h chain_ws_slots sizes the slots)
template <class M, class = void>
struct WsStashOf {
  static constexpr bool value = false;
};
template <class M>
struct WsStashOf<M, std::void_t<decltype(M::kWsStash)>> {
  static constexpr bool value = M::kWsStash;
};

// AONE: bit r*NX+j set = A[r][j] is exactly 1 (a model's structural unit entries, within AMASK):
// such terms enter as additions, and the sums start from them.  Hux' is formed as A^T (P B) when
// A's columns are sparser than B's (the unicycle: A = I + two entries in column 2), else as
// B^T (P A).
__host__ __device__ constexpr int popc64(unsigned long long v) { return v ? (int)(v & 1ull) + popc64(v >> 1) : 0; }
template <int NX, int NU>
__host__ __device__ constexpr unsigned long long col_mask(unsigned long long mask, int ncol, int j, int nrow) {
  unsigned long long r = 0;
  for (int m = 0; m < nrow; ++m) r |= ((mask >> (m * ncol + j)) & 1ull) << m;
  return r;
}
template <int NX, int NU, unsigned long long AMASK, unsigned long long BMASK>
__host__ __device__ constexpr bool hux_by_atpb() {
  int bt = 0, at = 0;
  for (int l = 0; l < NU; ++l)
    for (int j = 0; j < NX; ++j) {
      bt += popc64(col_mask<NX, NU>(BMASK, NU, l, NX));
      at += popc64(col_mask<NX, NU>(AMASK, NX, j, NX));
    }
  return at < bt;
}

template <int NX, int NU, unsigned long long AMASK, unsigned long long BMASK, bool DEC = false, bool SREORD = false,
          unsigned long long AONE = 0>
__device__ __forceinline__ bool riccati_step(const double* Hd, const double* gp, const double* A, const double* Bm,
                                             const double* c, const double* P, const double* p, double* Pn,
                                             double* pn, Fac<NX, NU>& f, const double* Pown = nullptr,
                                             const double* vpre = nullptr) {
  static_assert(!DEC || SREORD, "DEC takes s in the SREORD order");
  static_assert((AONE & ~AMASK) == 0, "unit entries must be inside AMASK");
  constexpr int NZ = NX + NU;
  static_assert(NU == 1 || NU == 2, "NU must be 1 or 2");
  auto Pm = [&](int i, int j) { return P[symix(i, j, NX)]; };
  double Hxx[NX * NX], Hux[NU * NX], Huu[NU * NU];
  if constexpr (DEC) {
#pragma unroll
    for (int l = 0; l < NU; ++l) {
#pragma unroll
      for (int j = 0; j < NX; ++j) Hux[l * NX + j] = Hd[symix(j, NX + l, NZ)];
#pragma unroll
      for (int n = l; n < NU; ++n) Huu[l * NU + n] = Hd[symix(NX + l, NX + n, NZ)];
    }
  } else {
  // PA = P A, PB = P B.  Sums start from their first structural term (a product, not an
  // fma into 0.0): a model's structural ones then fold away (P * 1.0 == P exactly, while
  // fma(P, 1.0, 0.0) must be kept for the sign of zero).
  double PA[NX * NX], PB[NX * NU];
#pragma unroll
  for (int r = 0; r < NX; ++r) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double acc = 0.0;
      bool first = true;
#pragma unroll
      for (int m = 0; m < NX; ++m)  // unit terms first (additions), then the others as FMAs
        if (AONE & (1ull << (m * NX + j))) {
          acc = first ? Pm(r, m) : acc + Pm(r, m);
          first = false;
        }
#pragma unroll
      for (int m = 0; m < NX; ++m)
        if ((AMASK & ~AONE) & (1ull << (m * NX + j))) {
          acc = first ? Pm(r, m) * A[m * NX + j] : fma(Pm(r, m), A[m * NX + j], acc);
          first = false;
        }
      PA[r * NX + j] = acc;
    }
#pragma unroll
    for (int l = 0; l < NU; ++l) {
      double acc = 0.0;
      bool first = true;
#pragma unroll
      for (int m = 0; m < NX; ++m)
        if (BMASK & (1ull << (m * NU + l))) {
          acc = first ? Pm(r, m) * Bm[m * NU + l] : fma(Pm(r, m), Bm[m * NU + l], acc);
          first = false;
        }
      PB[r * NU + l] = acc;
    }
  }
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = i; j < NX; ++j) {
      double acc = Hd[symix(i, j, NZ)];
#pragma unroll
      for (int m = 0; m < NX; ++m)
        if (AMASK & (1ull << (m * NX + i))) acc = fma(A[m * NX + i], PA[m * NX + j], acc);
      Hxx[i * NX + j] = acc;
    }
  constexpr bool kAtPB = hux_by_atpb<NX, NU, AMASK, BMASK>();
#pragma unroll
  for (int l = 0; l < NU; ++l) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double acc = Hd[symix(j, NX + l, NZ)];
      if constexpr (kAtPB) {  // Hux'[l][j] = Hd + sum_m A[m][j] (P B)[m][l]
#pragma unroll
        for (int m = 0; m < NX; ++m)
          if (AONE & (1ull << (m * NX + j))) acc += PB[m * NU + l];
#pragma unroll
        for (int m = 0; m < NX; ++m)
          if ((AMASK & ~AONE) & (1ull << (m * NX + j))) acc = fma(A[m * NX + j], PB[m * NU + l], acc);
      } else {  // Hd + sum_m B[m][l] (P A)[m][j]
#pragma unroll
        for (int m = 0; m < NX; ++m)
          if (BMASK & (1ull << (m * NU + l))) acc = fma(Bm[m * NU + l], PA[m * NX + j], acc);
      }
      Hux[l * NX + j] = acc;
    }
#pragma unroll
    for (int n = l; n < NU; ++n) {
      double acc = Hd[symix(NX + l, NX + n, NZ)];
#pragma unroll
      for (int m = 0; m < NX; ++m)
        if (BMASK & (1ull << (m * NU + l))) acc = fma(Bm[m * NU + l], PB[m * NU + n], acc);
      Huu[l * NU + n] = acc;
    }
  }
  }  // !DEC
  double s[NX], gx[NX], gu[NU];
  if constexpr (DEC) {
#pragma unroll
    for (int i = 0; i < NX; ++i) s[i] = vpre[i] + p[i];
  } else if constexpr (SREORD) {
#pragma unroll
    for (int i = 0; i < NX; ++i) s[i] = riccati_pc_row<NX>(P, c, i) + p[i];
  } else {
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      double acc = p[i];
#pragma unroll
      for (int m = 0; m < NX; ++m) acc = fma(Pm(i, m), c[m], acc);
      s[i] = acc;
    }
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    double acc = gp[i];
#pragma unroll
    for (int m = 0; m < NX; ++m)
      if (AMASK & (1ull << (m * NX + i))) acc = fma(A[m * NX + i], s[m], acc);
    gx[i] = acc;
  }
#pragma unroll
  for (int l = 0; l < NU; ++l) {
    double acc = gp[NX + l];
#pragma unroll
    for (int m = 0; m < NX; ++m)
      if (BMASK & (1ull << (m * NU + l))) acc = fma(Bm[m * NU + l], s[m], acc);
    gu[l] = acc;
  }
  bool ok;
  if constexpr (NU == 1) {
    const double d0 = Huu[0];
    ok = d0 > 0.0;
    f.r0 = rcp64(d0);
    f.r1 = 0.0;
    f.t = 0.0;
    f.g0 = gu[0];
    f.g1 = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      f.h0[j] = Hux[j];
      f.h1[j] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const double ri = f.r0 * f.h0[i];
#pragma unroll
      for (int j = i; j < NX; ++j) Pn[symix(i, j, NX)] = DEC ? Pown[symix(i, j, NX)] : fma(-ri, f.h0[j], Hxx[i * NX + j]);
      pn[i] = fma(-ri, f.g0, gx[i]);
    }
  } else {
    const double a = Huu[0], b = Huu[1], d = Huu[3];
    const double det = fma(a, d, -b * b);
    ok = (a > 0.0) && (det > 0.0);
    const double ra = rcp64(a), rdet = rcp64(det);  // independent
    f.r0 = ra;
    f.t = b * ra;
    f.r1 = a * rdet;  // 1 / (d - b^2/a)
    f.g0 = gu[0];
    f.g1 = fma(-f.t, gu[0], gu[1]);
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      f.h0[j] = Hux[j];
      f.h1[j] = fma(-f.t, Hux[j], Hux[NX + j]);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const double r0i = f.r0 * f.h0[i], r1i = f.r1 * f.h1[i];
#pragma unroll
      for (int j = i; j < NX; ++j)
        Pn[symix(i, j, NX)] = DEC ? Pown[symix(i, j, NX)] : fma(-r1i, f.h1[j], fma(-r0i, f.h0[j], Hxx[i * NX + j]));
      pn[i] = fma(-r1i, f.g1, fma(-r0i, f.g0, gx[i]));
    }
  }
  return ok;
}

// The DEC step split in two: dec_prefactor (off the chain: the factors, which need no p) and
// dec_vector_step (on the chain: s and p_k); P_k is the stored one.
template <int NX, int NU>
__device__ __forceinline__ bool dec_prefactor(const double* Hd, Fac<NX, NU>& f) {
  constexpr int NZ = NX + NU;
  if constexpr (NU == 1) {
    const double d0 = Hd[symix(NX, NX, NZ)];
    f.r0 = rcp64(d0);
    f.r1 = 0.0;
    f.t = 0.0;
    f.g1 = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      f.h0[j] = Hd[symix(j, NX, NZ)];
      f.h1[j] = 0.0;
    }
    return d0 > 0.0;
  } else {
    const double a = Hd[symix(NX, NX, NZ)], b = Hd[symix(NX, NX + 1, NZ)], d = Hd[symix(NX + 1, NX + 1, NZ)];
    const double det = fma(a, d, -b * b);
    const double ra = rcp64(a), rdet = rcp64(det);
    f.r0 = ra;
    f.t = b * ra;
    f.r1 = a * rdet;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      f.h0[j] = Hd[symix(j, NX, NZ)];
      f.h1[j] = fma(-f.t, Hd[symix(j, NX, NZ)], Hd[symix(j, NX + 1, NZ)]);
    }
    return (a > 0.0) && (det > 0.0);
  }
}

// On a decoupled stage B = 0 and Hux' = 0 exactly, so gu = gp_u and p_k = gx = gp_x + A^T s
// (s = P_{k+1} c + p_{k+1}, vpre = P_{k+1} c): the full step's extra terms, B^T s and
// -(L^{-1} Hux')^T D^{-1} L^{-1} gu', are exact zeros (they could change only the sign of an
// exact zero), so the chain carries s and gx alone.
template <int NX, int NU, unsigned long long AMASK, unsigned long long BMASK>
__device__ __forceinline__ void dec_vector_step(const double* gp, const double* A, const double* Bm, const double* vpre,
                                                const double* p, double* pn, Fac<NX, NU>& f) {
  (void)Bm;
  double s[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) s[i] = vpre[i] + p[i];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    double acc = gp[i];
#pragma unroll
    for (int m = 0; m < NX; ++m)
      if (AMASK & (1ull << (m * NX + i))) acc = fma(A[m * NX + i], s[m], acc);
    pn[i] = acc;
  }
  f.g0 = gp[NX];
  if constexpr (NU == 2) f.g1 = fma(-f.t, gp[NX], gp[NX + 1]);
}

// The inertia verdict of a step from its factors (off the chain, all lanes at once): Huu' is
// positive definite iff its LDL^T pivots are -- r0 = 1/d0 and (NU = 2) r1 = d0/det positive and
// finite.  The same answer as the step's own test (d0 > 0, det > 0) but where a reciprocal
// overflows (a pivot below ~1e-308) or is NaN, which the test reads as indefinite too.
template <int NX, int NU>
__device__ __forceinline__ bool fac_ok(const Fac<NX, NU>& f) {
  const bool a = f.r0 > 0.0 && f.r0 < INFINITY;
  if constexpr (NU == 1) return a;
  return a && f.r1 > 0.0 && f.r1 < INFINITY;
}

// K = -Huu'^{-1} Hux', kf = -Huu'^{-1} gu' from the LDL^T data (off the critical path).
template <int NX, int NU>
__device__ __forceinline__ void riccati_gains(const Fac<NX, NU>& f, double* K, double* kf) {
  if constexpr (NU == 1) {
#pragma unroll
    for (int j = 0; j < NX; ++j) K[j] = -f.r0 * f.h0[j];
    kf[0] = -f.r0 * f.g0;
  } else {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const double y1 = f.r1 * f.h1[j];
      K[NX + j] = -y1;
      K[j] = -fma(f.r0, f.h0[j], -f.t * y1);
    }
    const double z1 = f.r1 * f.g1;
    kf[1] = -z1;
    kf[0] = -fma(f.r0, f.g0, -f.t * z1);
  }
}

}  // namespace mpcx
