// collectives.h -- lane-group collectives of the fused solve kernel (gfx950, all VALU).
//
// A lane group = G contiguous lanes (G = 16/32/64) holding one MPC instance, lane k =
// shooting node k.  Neighbour moves are DPP wave shifts; all-reduces are DPP within a
// 16-lane row (quad_perm xor1, quad_perm xor2, row_half_mirror, row_mirror) followed by
// v_permlane16_swap / v_permlane32_swap across rows.  Every combine is symmetric (a+b on
// one lane, b+a on its partner), so all lanes of a group end with bit-identical results
// and take identical control decisions.
#pragma once
#include <hip/hip_runtime.h>

#include <utility>

namespace mpcx {

// v_mov_b32_dpp with bound_ctrl: lanes whose source is out of range read 0, so the
// destination needs no initialising move (update_dpp with an explicit `old` costs one
// extra v_mov per 32-bit half -- on the sequential Riccati chain that is ~10 % of a step).
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffLL), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kQuadXor1 = 0xb1, kQuadXor2 = 0x4e, kHalfMirror = 0x141, kMirror = 0x140;
constexpr int kWaveShl1 = 0x130, kWaveShr1 = 0x138;

struct Pair {
  double a, b;
};
// the two 16-lane rows of each 32-lane half (xor 16), in a fixed order
__device__ __forceinline__ Pair rows16(double v) {
  const long long x = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap((int)(x & 0xffffffffLL), (int)(x & 0xffffffffLL), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((int)(x >> 32), (int)(x >> 32), false, false);
  return {__longlong_as_double(((long long)hi[0] << 32) | (unsigned int)lo[0]),
          __longlong_as_double(((long long)hi[1] << 32) | (unsigned int)lo[1])};
}
// the two 32-lane halves of the wave (xor 32), in a fixed order
__device__ __forceinline__ Pair halves32(double v) {
  const long long x = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((int)(x & 0xffffffffLL), (int)(x & 0xffffffffLL), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((int)(x >> 32), (int)(x >> 32), false, false);
  return {__longlong_as_double(((long long)hi[0] << 32) | (unsigned int)lo[0]),
          __longlong_as_double(((long long)hi[1] << 32) | (unsigned int)lo[1])};
}

// max / min of doubles that are never signalling NaNs -- every value of the solve loop is an
// arithmetic result, a DPP/permlane copy of one or a load of one -- as the bare v_max_f64 /
// v_min_f64.  LLVM's fmax/fmin must first quiet each operand it cannot prove quiet (a
// `v_max_f64 x, x` per DPP-moved, loaded or |.|-modified operand: 229 of the config-2 kernel's
// 404 v_max_f64); the instruction's result for quiet NaNs and numbers is the same.
__device__ __forceinline__ double qmax(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double qmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// max(a, |b|) with the abs source modifier
__device__ __forceinline__ double qmax_abs(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

struct OpSum {
  __device__ static double f(double a, double b) { return a + b; }
};
struct OpMax {
  __device__ static double f(double a, double b) { return qmax(a, b); }
};
struct OpMin {
  __device__ static double f(double a, double b) { return qmin(a, b); }
};

// Groups wider than a wavefront (G = 128 / 256: horizons N >= 64) span G/64 waves of one
// workgroup.  Their collectives finish through LDS: every exchange writes the current
// slot of a 2-slot buffer, passes one workgroup barrier and flips the slot, so the next
// exchange can never overwrite values a slower wave is still reading (a wave can be at
// most one barrier ahead).  All waves execute the same sequence of exchanges because
// every branch around them is group-uniform.
constexpr int kXchStride = 48;  // doubles per wave per slot (>= NP + NX and NX^2 + NX of the largest model)
template <int G>
struct XWave {
  static constexpr int W = G > 64 ? G / 64 : 1;
  double* buf;  // [2][W][kXchStride] in LDS (unused when W == 1)
  int slot;
  __device__ __forceinline__ double* cur() const { return buf + slot * (W * kXchStride); }
  __device__ __forceinline__ double* prev() const { return buf + (slot ^ 1) * (W * kXchStride); }
  __device__ __forceinline__ void sync() {
    __syncthreads();
    slot ^= 1;
  }
};

template <int G, class Op>
__device__ __forceinline__ double greduce(double v, XWave<G>& xw) {
  v = Op::f(v, dpp<kQuadXor1>(v));
  v = Op::f(v, dpp<kQuadXor2>(v));
  v = Op::f(v, dpp<kHalfMirror>(v));
  v = Op::f(v, dpp<kMirror>(v));
  if (G >= 32) {
    const Pair p = rows16(v);
    v = Op::f(p.a, p.b);
  }
  if (G >= 64) {
    const Pair p = halves32(v);
    v = Op::f(p.a, p.b);
  }
  if constexpr (G > 64) {
    constexpr int W = G / 64;
    double* b = xw.cur();
    if ((threadIdx.x & 63) == 0) b[(threadIdx.x >> 6) * kXchStride] = v;
    __syncthreads();
    double r = b[0];
#pragma unroll
    for (int w = 1; w < W; ++w) r = Op::f(r, b[w * kXchStride]);  // same order on every wave
    xw.slot ^= 1;
    return r;
  }
  return v;
}
// Several group reductions at once (OPS: 0 sum, 1 max, 2 min, 3 "all" of 0/1 flags, one per
// value): the in-wave DPP chains as greduce's -- for "all" one ballot when the group fills the
// wave -- and for groups wider than a wave ONE LDS exchange and barrier for all of them (a barrier
// is the expensive part there: the waves of a group meet at every one).
__device__ __forceinline__ double op_apply(int op, double a, double b) {  // op a compile-time constant after unrolling
  return op == 0 ? a + b : op == 1 ? qmax(a, b) : qmin(a, b);
}
template <int G>
__device__ __forceinline__ double wreduce(int op, double v) {  // over the group's lanes inside one wave
  if (G >= 64 && op == 3) return __ballot(!(v > 0.5)) == 0 ? 1.0 : 0.0;  // every (active) lane holds 1
  v = op_apply(op, v, dpp<kQuadXor1>(v));
  v = op_apply(op, v, dpp<kQuadXor2>(v));
  v = op_apply(op, v, dpp<kHalfMirror>(v));
  v = op_apply(op, v, dpp<kMirror>(v));
  if (G >= 32) {
    const Pair p = rows16(v);
    v = op_apply(op, p.a, p.b);
  }
  if (G >= 64) {
    const Pair p = halves32(v);
    v = op_apply(op, p.a, p.b);
  }
  return v;
}
template <int G, int... OPS>
__device__ __forceinline__ void greduce_n(double* v, XWave<G>& xw) {
  constexpr int n = sizeof...(OPS);
  constexpr int ops[n] = {OPS...};
  static_assert(n <= kXchStride, "exchange slot");
#pragma unroll
  for (int i = 0; i < n; ++i) v[i] = wreduce<G>(ops[i], v[i]);
  if constexpr (G > 64) {
    constexpr int W = G / 64;
    double* b = xw.cur();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int i = 0; i < n; ++i) b[(threadIdx.x >> 6) * kXchStride + i] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < n; ++i) {
      double r = b[i];
#pragma unroll
      for (int w = 1; w < W; ++w) r = op_apply(ops[i], r, b[w * kXchStride + i]);  // same order on every wave
      v[i] = r;
    }
    xw.slot ^= 1;
  }
}

template <int G>
__device__ __forceinline__ double gsum(double v, XWave<G>& xw) {
  return greduce<G, OpSum>(v, xw);
}
template <int G>
__device__ __forceinline__ double gmax(double v, XWave<G>& xw) {
  return greduce<G, OpMax>(v, xw);
}
template <int G>
__device__ __forceinline__ double gmin(double v, XWave<G>& xw) {
  return greduce<G, OpMin>(v, xw);
}
// Group tests by ballot: true on every lane of the group iff c holds on all of its (active) lanes.
// A threshold test on a group max -- max_k e_k <= t -- is the group test of e_k <= t (max is exact),
// so the solve loop's convergence, acceptable-level and barrier tests need no max reduction (a
// 5-6 level DPP/permlane chain of ~25 instructions) but one ballot.  L = lanes of one instance in
// the wave: G, or 64 for a replicated 32-lane group (kernels.h R = 2), whose test is wave-uniform.
template <int G, int L = G>
__device__ __forceinline__ bool gall(bool c, XWave<G>& xw) {
  if constexpr (G > 64) {  // a ballot per wave, one exchange
    double t = c ? 1.0 : 0.0;
    greduce_n<G, 3>(&t, xw);
    return t > 0.5;
  } else {
    const unsigned long long f = __ballot(!c);  // lanes where c fails
    if constexpr (L >= 64) {
      return f == 0;
    } else {
      const int sh = (int)(threadIdx.x & 63) & ~(G - 1);
      return ((f >> sh) & ((1ull << G) - 1)) == 0;
    }
  }
}
template <int G, int L = G>
__device__ __forceinline__ bool gany(bool c, XWave<G>& xw) {
  return !gall<G, L>(!c, xw);
}

// value of lane k+1 / k-1 (whole-wave DPP shift; groups are contiguous and the lanes
// that would read across a group boundary never use the value)
__device__ __forceinline__ double from_next(double v) { return dpp<kWaveShl1>(v); }
__device__ __forceinline__ double from_prev(double v) { return dpp<kWaveShr1>(v); }

// Partner of level d (1, 2, 4, 8, 16, 32) of a wave-wide inclusive prefix scan, as DPP moves
// (VALU, no LDS crossbar round trip): row_shr:d inside each 16-lane row for d <= 8, then
// row_bcast:15 (lane 16r-1 to row r) and row_bcast:31 (lane 31 to rows 2, 3).  After the
// in-row levels lane l holds the row's prefix up to l; the broadcasts carry the previous
// rows' total in.  scan_takes<d>(kw) says whether the lane at wave position kw combines.
template <int D>
__device__ __forceinline__ double scan_partner(double v) {
  static_assert(D == 1 || D == 2 || D == 4 || D == 8 || D == 16 || D == 32, "scan level");
  return dpp<D <= 8 ? 0x110 + D : D == 16 ? 0x142 : 0x143>(v);
}
template <int D>
__device__ __forceinline__ bool scan_takes(int kw) {
  return D <= 8 ? (kw & 15) >= D : (kw & D) != 0;
}

// value of lane `src` of the wave (any lane; ds_bpermute through the LDS crossbar, no LDS memory)
__device__ __forceinline__ double from_lane(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b & 0xffffffffLL));
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// out[i] = v[i] of node k+1 for node-parallel phases; for multi-wave groups lane 63 of
// wave w receives lane 0 of wave w+1 through LDS.
template <int G, int n>
__device__ __forceinline__ void group_next(const double* v, double* out, XWave<G>& xw) {
#pragma unroll
  for (int i = 0; i < n; ++i) out[i] = from_next(v[i]);
  if constexpr (G > 64) {
    constexpr int W = G / 64;
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    double* b = xw.cur();
    if (ln == 0 && wv > 0)
#pragma unroll
      for (int i = 0; i < n; ++i) b[(wv - 1) * kXchStride + i] = v[i];
    __syncthreads();
    if (ln == 63 && wv < W - 1)
#pragma unroll
      for (int i = 0; i < n; ++i) out[i] = b[wv * kXchStride + i];
    xw.slot ^= 1;
  }
}

// acc[i] += sum_j M[i][j] w[j] (j ascending: the fma order of a plain loop) for an NX x NX matrix
// held as mA = M[r], mB = M[16 + r] on row lane r (NX = 4, 5): ONE asm statement behind ONE s_nop 1
// (round 5 had an s_nop 1 before each of the NX^2 FMAs: the VALU-write -> DPP-read hazard only concerns
// mA / mB, which the caller loads from LDS and nothing inside the block writes).  The accumulators
// are interleaved (j outer, i inner); each one still sums j ascending, so the bits are the plain loop's.
template <int NX>
__device__ __forceinline__ void matvec_bcast(double* acc, const double* w, double mA, double mB) {
  static_assert(NX == 4 || NX == 5, "row-broadcast mat-vec: NX = 4 or 5 (two row registers)");
  if constexpr (NX == 4) {
    asm volatile(
        "s_nop 1\n\t"  // covers a VALU write of mA / mB just before (none is written inside)
        "v_fmac_f64_dpp %0, %8, %4 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %8, %4 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %4 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %4 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %8, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %8, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %5 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %5 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %8, %6 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %8, %6 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %6 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %6 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %8, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %8, %7 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %7 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %7 row_newbcast:15 row_mask:0xf bank_mask:0xf"
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
        : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(mA), "v"(mB));
  } else {
    asm volatile(
        "s_nop 1\n\t"  // covers a VALU write of mA / mB just before (none is written inside)
        "v_fmac_f64_dpp %0, %10, %5 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %10, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %10, %5 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %10, %5 row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %11, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %10, %6 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %10, %6 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %10, %6 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %11, %6 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %11, %6 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %10, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %10, %7 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %10, %7 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %11, %7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %11, %7 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %10, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %10, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %10, %8 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %11, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %11, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %10, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %10, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %10, %9 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %11, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %11, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4])
        : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(mA), "v"(mB));
  }
}

// 1/x to full fp64 accuracy: v_rcp_f64 + two Newton steps (no IEEE division sequence
// on the sequential critical path)
__device__ __forceinline__ double rcp64(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

}  // namespace mpcx
