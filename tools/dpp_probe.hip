// dpp_probe.hip -- issue cost of the row chain's instruction kinds at one wave per SIMD (the solve
// kernel's occupancy): cycles per instruction of 64-long sequences, dependent (one accumulator) and
// independent (four), of v_fmac_f64, v_fmac_f64_dpp row_newbcast (with and without s_nop 1),
// v_mov_b64_dpp, v_mov_b32_dpp, v_rcp_f64 and a ds_read_b128 round trip.  s_memtime (shader
// clock) around each sequence; one wave per CU.  Build and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 tools/dpp_probe.hip -o tools/dpp_probe && tools/dpp_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP4(x) x x x x
#define REP16(x) REP4(x) REP4(x) REP4(x) REP4(x)
#define REP64(x) REP16(x) REP16(x) REP16(x) REP16(x)

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ __launch_bounds__(64) void probe(double* out, unsigned long long* cyc) {
  __shared__ double lds[1024];
  const int t = threadIdx.x;
  double a = 1.0 + t * 1e-3, b = 0.999, c0 = 0.1 * t, c1 = 0.2, c2 = 0.3, c3 = 0.4;
  for (int i = t; i < 1024; i += 64) lds[i] = i;
  __syncthreads();
  unsigned long long T[16];
  int n = 0;
  // A: dependent v_fmac_f64
  T[n++] = now();
  asm volatile(REP64("v_fmac_f64 %0, %1, %2\n\t") : "+v"(c0) : "v"(a), "v"(b));
  T[n++] = now();
  // B: independent v_fmac_f64 (four accumulators)
  asm volatile(REP16("v_fmac_f64 %0, %4, %5\n\tv_fmac_f64 %1, %4, %5\n\tv_fmac_f64 %2, %4, %5\n\tv_fmac_f64 %3, %4, %5\n\t")
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(a), "v"(b));
  T[n++] = now();
  // C: dependent v_fmac_f64_dpp row_newbcast (source not written: no nop needed)
  asm volatile(REP64("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t")
               : "+v"(c0) : "v"(a), "v"(b));
  T[n++] = now();
  // D: independent v_fmac_f64_dpp
  asm volatile(REP16("v_fmac_f64_dpp %0, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %4, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %2, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %3, %4, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t")
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(a), "v"(b));
  T[n++] = now();
  // E: s_nop 1 + dependent v_fmac_f64_dpp
  asm volatile(REP64("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t")
               : "+v"(c0) : "v"(a), "v"(b));
  T[n++] = now();
  // F: v_mov_b64_dpp (independent)
  double m0, m1, m2, m3;
  asm volatile(REP16("v_mov_b64_dpp %0, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %2, %4 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %3, %4 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t")
               : "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(m3) : "v"(a));
  T[n++] = now();
  // G: v_mov_b32_dpp (independent)
  int i0, i1, i2, i3, ia = t;
  asm volatile(REP16("v_mov_b32_dpp %0, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %1, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %2, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b32_dpp %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t")
               : "=&v"(i0), "=&v"(i1), "=&v"(i2), "=&v"(i3) : "v"(ia));
  T[n++] = now();
  // H: dependent v_rcp_f64
  double r = a;
  asm volatile(REP64("v_rcp_f64 %0, %0\n\t") : "+v"(r));
  T[n++] = now();
  // I: v_mul_f64 dependent (VOP3 FP64)
  double mm = a;
  asm volatile(REP64("v_mul_f64 %0, %0, %1\n\t") : "+v"(mm) : "v"(b));
  T[n++] = now();
  // J: v_add_u32 independent (32-bit VALU)
  int u0 = t, u1 = t, u2 = t, u3 = t;
  asm volatile(REP16("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4\n\t")
               : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(ia));
  T[n++] = now();
  // K: 16 ds_read_b128 round trips (load, wait, dependent address)
  int addr = t * 16;
  for (int k = 0; k < 16; ++k) {
    double2 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    addr = ((int)v.x & 63) * 16;
  }
  T[n++] = now();
  // L: v_cndmask_b32 independent
  asm volatile(REP16("v_cndmask_b32 %0, %0, %4, vcc\n\tv_cndmask_b32 %1, %1, %4, vcc\n\tv_cndmask_b32 %2, %2, %4, vcc\n\tv_cndmask_b32 %3, %3, %4, vcc\n\t")
               : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(ia));
  T[n++] = now();
  // M: chain through the DPP SOURCE: each fmac_dpp broadcasts the previous result (s_nop 1 between)
  double x = a, z = b;
  asm volatile(REP16("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "s_nop 1\n\tv_fmac_f64_dpp %1, %0, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "s_nop 1\n\tv_fmac_f64_dpp %1, %0, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t")
               : "+v"(x), "+v"(z) : "v"(b));
  T[n++] = now();
  // N: rcp64 chain (v_rcp_f64 + two Newton steps), each on the previous result
  double q = a;
  for (int k = 0; k < 16; ++k) {
    asm volatile(
        "v_rcp_f64 %1, %0\n\t"
        "v_fma_f64 %2, -%0, %1, 1.0\n\t"
        "v_fma_f64 %1, %1, %2, %1\n\t"
        "v_fma_f64 %2, -%0, %1, 1.0\n\t"
        "v_fma_f64 %0, %1, %2, %1"
        : "+v"(q), "=&v"(m0), "=&v"(m1));
  }
  T[n++] = now();
  // O: dependent v_fmac_f64 chain with a 2-instruction gap filled by independent work (latency probe)
  asm volatile(REP16("v_fmac_f64 %0, %4, %5\n\tv_fmac_f64 %1, %4, %5\n\tv_fmac_f64 %0, %4, %5\n\tv_fmac_f64 %1, %4, %5\n\t")
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(a), "v"(b));
  T[n++] = now();
  if (t == 0)
    for (int i = 0; i + 1 < n; ++i) cyc[blockIdx.x * 16 + i] = T[i + 1] - T[i];
  out[blockIdx.x * 64 + t] = x + z + q + c0 + c1 + c2 + c3 + m0 + m1 + m2 + m3 + r + mm + i0 + i1 + i2 + i3 + u0 + u1 + u2 + u3 + addr;
}

int main() {
  const int blocks = 256;
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * 64 * sizeof(double));
  hipMalloc(&cyc, blocks * 16 * sizeof(unsigned long long));
  hipMemset(cyc, 0, blocks * 16 * sizeof(unsigned long long));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, out, cyc);
  hipDeviceSynchronize();
  unsigned long long h[blocks * 16];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"fmac_f64 dependent",     "fmac_f64 independent x4", "fmac_f64_dpp dependent",
                         "fmac_f64_dpp indep x4",  "s_nop1+fmac_f64_dpp dep", "mov_b64_dpp indep x4",
                         "mov_b32_dpp indep x4",   "rcp_f64 dependent",       "mul_f64 dependent",
                         "add_u32 indep x4",       "ds_read_b128 round trip", "cndmask_b32 indep x4",
                         "nop+fmac_dpp chained through the dpp source", "rcp64 (rcp + 2 Newton) chained",
                         "fmac_f64 2-chain interleaved"};
  const double per[] = {64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 16, 64, 64, 16, 64};
  printf("{");
  for (int i = 0; i < 15; ++i) {
    double s = 0;
    for (int b = 0; b < blocks; ++b) s += h[b * 16 + i];
    printf("%s\"%s\": %.2f", i ? ", " : "", names[i], s / blocks / per[i]);
  }
  printf("}\n");
  return 0;
}
