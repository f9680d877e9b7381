// mfma_f64_probe.hip -- lane layouts and dependent-chain latencies of the FP64 MFMA instructions on
// gfx950 (the Riccati chain design question: can a 4x4x4 / 16x16x4 f64 MFMA replace the one-lane
// step?).  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_probe.hip -o tools/mfma_f64_probe
// Prints JSON: for each instruction, which (A lane, B lane) pairs feed each D element, and the
// cycles (s_memtime) per MFMA of a dependent chain D -> C and D -> B.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

// D lane/reg contents when A = one-hot at lane ta (value 1), B = one-hot at lane tb (value 1), C = 0
__global__ void probe4(int ta, int tb, double* out) {
  const int l = threadIdx.x;
  const double a = l == ta ? 1.0 : 0.0, b = l == tb ? 1.0 : 0.0;
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}
__global__ void probe16(int ta, int tb, double* out) {
  const int l = threadIdx.x;
  const double a = l == ta ? 1.0 : 0.0, b = l == tb ? 1.0 : 0.0;
  d4 c = {0.0, 0.0, 0.0, 0.0};
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[r * 64 + l] = d[r];
}

// dependent chains: kind 0 = D feeds C (accumulate), kind 1 = D feeds the B operand
template <int KIND>
__global__ void lat4(double* out, long long* cyc, int n) {
  const int l = threadIdx.x;
  double a = 1e-3 * (l + 1), b = 1.0 + 1e-4 * l, c = 0.0;
  const long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i += 16) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {  // unrolled: no loop branch between the dependent operations
      const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
      if (KIND == 0) c = d;
      else b = d;
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  out[l] = c + b;
  if (l == 0) *cyc = t1 - t0;
}
template <int KIND>
__global__ void lat16(double* out, long long* cyc, int n) {
  const int l = threadIdx.x;
  double a = 1e-3 * (l + 1), b = 1.0 + 1e-4 * l;
  d4 c = {0.0, 0.0, 0.0, 0.0};
  const long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i += 16) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
      if (KIND == 0) c = d;
      else b = d[0];
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  out[l] = c[0] + c[1] + c[2] + c[3] + b;
  if (l == 0) *cyc = t1 - t0;
}
// reference: a dependent chain of v_fma_f64 (one wave), and of independent ones (issue rate)
__global__ void indfma(double* out, long long* cyc, int n) {
  const int l = threadIdx.x;
  double a = 1.0 + 1e-9 * l, c[8];
  for (int j = 0; j < 8; ++j) c[j] = 1e-3 * j;
  const long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i += 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(a, c[j], 1e-3);  // 8 independent chains: 4 ops per i
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(a, c[j], 1e-3);
  }
  const long long t1 = __builtin_readcyclecounter();
  double t = 0;
  for (int j = 0; j < 8; ++j) t += c[j];
  out[l] = t;
  if (l == 0) *cyc = (t1 - t0) / 8;  // cycles per n of these = per 8 instructions / 8
}
__global__ void latfma(double* out, long long* cyc, int n) {
  const int l = threadIdx.x;
  double a = 1.0 + 1e-9 * l, c = 0.0;
  const long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i += 16) {
#pragma unroll
    for (int u = 0; u < 16; ++u) c = fma(a, c, 1e-3);
  }
  const long long t1 = __builtin_readcyclecounter();
  out[l] = c;
  if (l == 0) *cyc = t1 - t0;
}

// issue cost of cross-lane moves of a double: 8 independent DPP row shifts (2 x v_mov_b32_dpp
// each) or v_permlane32_swap pairs per step
template <int KIND>
__global__ void xlane(double* out, long long* cyc, int n) {
  const int l = threadIdx.x;
  double c[8];
  for (int j = 0; j < 8; ++j) c[j] = 1e-3 * (l + j);
  const long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i += 2) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const long long b = __double_as_longlong(c[j]);
        int lo = (int)(b & 0xffffffffLL), hi = (int)(b >> 32);
        if (KIND == 0) {
          lo = __builtin_amdgcn_mov_dpp(lo, 0x111, 0xf, 0xf, true);
          hi = __builtin_amdgcn_mov_dpp(hi, 0x111, 0xf, 0xf, true);
        } else if (KIND == 2) {  // ds_bpermute from lane ^ 32 (the LDS crossbar, no LDS memory)
          lo = __builtin_amdgcn_ds_bpermute((l ^ 32) << 2, lo);
          hi = __builtin_amdgcn_ds_bpermute((l ^ 32) << 2, hi);
        } else {
          const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
          const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
          lo = a[0];
          hi = h[0];
        }
        c[j] = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
      }
  }
  const long long t1 = __builtin_readcyclecounter();
  double t = 0;
  for (int j = 0; j < 8; ++j) t += c[j];
  out[l] = t;
  if (l == 0) *cyc = (t1 - t0) / 8;  // per double moved
}

// v_rcp_f64 and its Newton refinements: out[3 i + m] = m Newton steps from v_rcp_f64 of x[i]
__global__ void rcp_probe(const double* x, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  double r = __builtin_amdgcn_rcp(v);
  out[3 * i] = r;
  r = fma(r, fma(-v, r, 1.0), r);
  out[3 * i + 1] = r;
  r = fma(r, fma(-v, r, 1.0), r);
  out[3 * i + 2] = r;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  double* d;
  long long* cyc;
  CK(hipMalloc(&d, 256 * sizeof(double)));
  CK(hipMalloc(&cyc, sizeof(long long)));
  std::vector<double> h(256);
  printf("{\n \"mfma_f64_4x4x4_4b\": [");
  // A lane ta and B lane tb contribute to D element (lane) iff out[lane] == 1
  bool first = true;
  for (int ta = 0; ta < 64; ++ta)
    for (int tb = 0; tb < 64; ++tb) {
      probe4<<<1, 64>>>(ta, tb, d);
      CK(hipMemcpy(h.data(), d, 64 * sizeof(double), hipMemcpyDeviceToHost));
      for (int l = 0; l < 64; ++l)
        if (h[l] != 0.0) {
          printf("%s[%d,%d,%d]", first ? "" : ",", ta, tb, l);
          first = false;
        }
    }
  printf("],\n \"mfma_f64_16x16x4\": [");
  first = true;
  for (int ta = 0; ta < 64; ++ta)
    for (int tb = 0; tb < 64; ++tb) {
      probe16<<<1, 64>>>(ta, tb, d);
      CK(hipMemcpy(h.data(), d, 256 * sizeof(double), hipMemcpyDeviceToHost));
      for (int r = 0; r < 4; ++r)
        for (int l = 0; l < 64; ++l)
          if (h[r * 64 + l] != 0.0) {
            printf("%s[%d,%d,%d,%d]", first ? "" : ",", ta, tb, l, r);
            first = false;
          }
    }
  printf("],\n");
  const int n = 4096;
  long long c;
  auto run = [&](void (*k)(double*, long long*, int), const char* name, bool last) -> int {
    k<<<1, 64>>>(d, cyc, n);
    CK(hipDeviceSynchronize());
    k<<<1, 64>>>(d, cyc, n);
    CK(hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost));
    printf(" \"%s_cycles_per_op\": %.2f%s\n", name, (double)c / n, last ? "" : ",");
    return 0;
  };
  if (run(lat4<0>, "lat4_d_to_c", false)) return 1;
  if (run(lat4<1>, "lat4_d_to_b", false)) return 1;
  if (run(lat16<0>, "lat16_d_to_c", false)) return 1;
  if (run(lat16<1>, "lat16_d_to_b", false)) return 1;
  if (run(latfma, "fma_f64_dep", false)) return 1;
  if (run(indfma, "fma_f64_indep_issue", false)) return 1;
  if (run(xlane<0>, "dpp_row_shift_per_double", false)) return 1;
  if (run(xlane<1>, "permlane32_swap_per_double", false)) return 1;
  if (run(xlane<2>, "ds_bpermute_xor32_per_double", false)) return 1;
  // relative error of v_rcp_f64 with 0 / 1 / 2 Newton steps over 2^20 inputs spread over 1e-12..1e12
  {
    const int m = 1 << 20;
    std::vector<double> hx(m), hr(3 * m);
    unsigned long long st = 88172645463325252ull;
    for (int i = 0; i < m; ++i) {
      st ^= st << 13;
      st ^= st >> 7;
      st ^= st << 17;
      const double u = (double)(st >> 11) / 9007199254740992.0;
      hx[i] = std::pow(10.0, -12.0 + 24.0 * u) * ((st & 1) ? 1.0 : -1.0);
    }
    double *dx, *dr;
    CK(hipMalloc(&dx, m * sizeof(double)));
    CK(hipMalloc(&dr, 3 * m * sizeof(double)));
    CK(hipMemcpy(dx, hx.data(), m * sizeof(double), hipMemcpyHostToDevice));
    rcp_probe<<<m / 256, 256>>>(dx, dr, m);
    CK(hipMemcpy(hr.data(), dr, 3 * m * sizeof(double), hipMemcpyDeviceToHost));
    double e[3] = {0, 0, 0};
    for (int i = 0; i < m; ++i)
      for (int k = 0; k < 3; ++k) e[k] = std::max(e[k], std::fabs(hr[3 * i + k] * hx[i] - 1.0));
    printf(" \"rcp_f64_max_rel_err\": [%.3e, %.3e, %.3e]\n", e[0], e[1], e[2]);
  }
  printf("}\n");
  return 0;
}
