// hbm_probe.hip -- streaming ceilings of one MI355X for the sweep's access mix (tools/, not product).
//   write-only, read-only and a 1:4.5 read:write stream (the rk4_sens ratio: 848 B read per
//   3840 B written per instance), all with 16-B per-lane accesses, >= 2 GB per pass so the
//   256 MiB Infinity Cache cannot hold it.  hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ void wr(double2* __restrict__ o, long n, double v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    o[i] = make_double2(v, v + i);
}
__global__ void rd(const double2* __restrict__ a, long n, double* out) {
  double s = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double2 x = a[i];
    s += x.x + x.y;
  }
  if (s == 1234.5) out[0] = s;
}
__global__ void wr_nt(double2* __restrict__ o, long n, double v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    __builtin_nontemporal_store(v, &o[i].x);
    __builtin_nontemporal_store(v + i, &o[i].y);
  }
}
__global__ void wr_flat(double2* __restrict__ o, long n, double v) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) o[i] = make_double2(v, v + i);
}
__global__ void wr8(double* __restrict__ o, long n, double v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) o[i] = v + i;
}
// the sweep's store pattern, write only: B instances (2 per lane), S stages, 24 fields.
// SoA: field row f*S... address ((k*24 + f) * B + b) -- rows B*8 bytes apart.
__global__ void sweep_soa(double* __restrict__ o, int B, int S) {
  const long b0 = 2 * ((long)blockIdx.x * blockDim.x + threadIdx.x);
  if (b0 >= B) return;
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int f = 0; f < 24; ++f)
      *reinterpret_cast<double2*>(o + ((long)k * 24 + f) * B + b0) = make_double2(k + f, b0);
}
// tiled: per stage, each wave's 128 instances x 24 fields are one contiguous 24 KB block.
__global__ void sweep_tiled(double* __restrict__ o, int B, int S) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long b0 = 2 * t;
  if (b0 >= B) return;
  const long tile = b0 / 128, lane2 = b0 % 128;
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int f = 0; f < 24; ++f)
      *reinterpret_cast<double2*>(o + (((long)k * (B / 128) + tile) * 24 + f) * 128 + lane2) = make_double2(k + f, b0);
}
// tile-major: each wave's whole output (S stages x 24 fields x 128) is one contiguous region
__global__ void sweep_tilemajor(double* __restrict__ o, int B, int S) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long b0 = 2 * t;
  if (b0 >= B) return;
  const long tile = b0 / 128, lane2 = b0 % 128;
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int f = 0; f < 24; ++f)
      *reinterpret_cast<double2*>(o + ((tile * S + k) * 24 + f) * 128 + lane2) = make_double2(k + f, b0);
}
// tiled with 64-instance tiles (8-B per lane, one instance per lane)
__global__ void sweep_tiled64(double* __restrict__ o, int B, int S) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long tile = b / 64, lane = b % 64;
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int f = 0; f < 24; ++f) o[(((long)k * (B / 64) + tile) * 24 + f) * 64 + lane] = k + f + b;
}
// the sweep's exact traffic without its arithmetic: tiled X/U loads, one 24-field record store
// per stage (tix layout of solver.hip), 64 instances per tile
__device__ __forceinline__ size_t ptix(int stage, int F, int i, long b, long T) {
  return (((size_t)stage * T + (b >> 6)) * F + i) * 64 + (b & 63);
}
__global__ void sweep_copy(const double* __restrict__ X, const double* __restrict__ U, double* __restrict__ J, int B,
                           int S) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long T = (B + 63) / 64;
  double x0 = X[ptix(0, 3, 0, b, T)], x1 = X[ptix(0, 3, 1, b, T)], x2 = X[ptix(0, 3, 2, b, T)];
  for (int k = 0; k < S; ++k) {
    const double n0 = X[ptix(k + 1, 3, 0, b, T)], n1 = X[ptix(k + 1, 3, 1, b, T)], n2 = X[ptix(k + 1, 3, 2, b, T)];
    const double u0 = U[ptix(k, 2, 0, b, T)], u1 = U[ptix(k, 2, 1, b, T)];
    const double base = x0 + x1 + x2 + u0 + u1;
#pragma unroll
    for (int f = 0; f < 24; ++f) J[ptix(k, 24, f, b, T)] = base + f;
    x0 = n0;
    x1 = n1;
    x2 = n2;
  }
}

// as sweep_copy, but the 24-field record is stored as 12 field pairs: lane writes 16 B
// (fields 2j, 2j+1) at ((stage*T + tile)*12 + j)*64 + lane, i.e. 1 KB per wave-instruction
template <bool NT>
__global__ void sweep_copy16(const double* __restrict__ X, const double* __restrict__ U, double* __restrict__ J, int B,
                             int S) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long T = (B + 63) / 64;
  double x0 = X[ptix(0, 3, 0, b, T)], x1 = X[ptix(0, 3, 1, b, T)], x2 = X[ptix(0, 3, 2, b, T)];
  typedef double v2d __attribute__((ext_vector_type(2)));
  v2d* J2 = reinterpret_cast<v2d*>(J);
  for (int k = 0; k < S; ++k) {
    const double n0 = X[ptix(k + 1, 3, 0, b, T)], n1 = X[ptix(k + 1, 3, 1, b, T)], n2 = X[ptix(k + 1, 3, 2, b, T)];
    const double u0 = U[ptix(k, 2, 0, b, T)], u1 = U[ptix(k, 2, 1, b, T)];
    const double base = x0 + x1 + x2 + u0 + u1;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      v2d v = {base + 2 * j, base + 2 * j + 1};
      v2d* p = &J2[ptix(k, 12, j, b, T)];
      if (NT) __builtin_nontemporal_store(v, p);
      else *p = v;
    }
    x0 = n0;
    x1 = n1;
    x2 = n2;
  }
}

// flat stage-parallel form: one thread per (instance, stage); block order = output order
// (stage-major, 4 tiles of one stage per 256-thread block), so the write front sweeps
// memory linearly as blocks are dispatched.  x_{k+1} is read by two threads (stages k, k+1).
template <int W, bool NT>
__global__ void sweep_flat(const double* __restrict__ X, const double* __restrict__ U, double* __restrict__ J, int B,
                           int S) {
  const long T = (B + 63) / 64;
  const long tpb = blockDim.x / 64;                 // tiles per block
  const long bps = (T + tpb - 1) / tpb;             // blocks per stage
  const int k = (int)(blockIdx.x / bps);
  const long b = (blockIdx.x % bps) * blockDim.x + threadIdx.x;
  if (k >= S || b >= B) return;
  const double x0 = X[ptix(k, 3, 0, b, T)], x1 = X[ptix(k, 3, 1, b, T)], x2 = X[ptix(k, 3, 2, b, T)];
  const double n0 = X[ptix(k + 1, 3, 0, b, T)], n1 = X[ptix(k + 1, 3, 1, b, T)], n2 = X[ptix(k + 1, 3, 2, b, T)];
  const double u0 = U[ptix(k, 2, 0, b, T)], u1 = U[ptix(k, 2, 1, b, T)];
  const double base = x0 + x1 + x2 + u0 + u1 + n0 * n1 * n2;
  if (W == 8) {
#pragma unroll
    for (int f = 0; f < 24; ++f) {
      if (NT) __builtin_nontemporal_store(base + f, &J[ptix(k, 24, f, b, T)]);
      else J[ptix(k, 24, f, b, T)] = base + f;
    }
  } else {
    typedef double v2d __attribute__((ext_vector_type(2)));
    v2d* J2 = reinterpret_cast<v2d*>(J);
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      v2d v = {base + 2 * j, base + 2 * j + 1};
      if (NT) __builtin_nontemporal_store(v, &J2[ptix(k, 12, j, b, T)]);
      else J2[ptix(k, 12, j, b, T)] = v;
    }
  }
}
// per element of `a`: 1 read, ~4.5 writes (9 writes per 2 reads)
__global__ void mix(const double2* __restrict__ a, double2* __restrict__ o, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double2 x = a[i];
    const int reps = (i & 1) ? 5 : 4;
    for (int r = 0; r < reps; ++r) o[(long)r * n + i] = make_double2(x.x + r, x.y - r);
  }
}

int main() {
  const long nw = (2L << 30) / 16;  // 2 GiB of double2
  double2 *a, *o;
  double* out;
  CK(hipMalloc(&a, nw * 16));
  CK(hipMalloc(&o, 5 * (nw / 4) * 16 + 16));
  CK(hipMalloc(&out, 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 8 * 4, block = 256;
  float ms;
  auto timeit = [&](auto launch, double bytes, const char* name) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 10; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"probe\": \"%s\", \"GBps\": %.1f, \"ms\": %.4f}\n", name, bytes / (ms / 10 * 1e-3) / 1e9, ms / 10);
  };
  timeit([&] { hipLaunchKernelGGL(wr, dim3(grid), dim3(block), 0, 0, a, nw, 1.0); }, nw * 16.0, "write 16B/lane");
  timeit([&] { hipLaunchKernelGGL(wr_nt, dim3(grid), dim3(block), 0, 0, a, nw, 1.0); }, nw * 16.0, "write nt 16B/lane");
  timeit([&] { hipLaunchKernelGGL(wr_flat, dim3((unsigned)((nw + 255) / 256)), dim3(block), 0, 0, a, nw, 1.0); },
         nw * 16.0, "write 16B/lane one element per thread");
  timeit([&] { hipLaunchKernelGGL(wr8, dim3(grid), dim3(block), 0, 0, (double*)a, 2 * nw, 1.0); }, nw * 16.0,
         "write 8B/lane");
  timeit([&] { hipLaunchKernelGGL(rd, dim3(grid), dim3(block), 0, 0, a, nw, out); }, nw * 16.0, "read 16B/lane");
  {
    const int Bs = 1 << 19, S = 20;
    double* ob;
    CK(hipMalloc(&ob, (long)Bs * S * 24 * 8));
    const double by = (double)Bs * S * 24 * 8;
    timeit([&] { hipLaunchKernelGGL(sweep_soa, dim3(Bs / 2 / 256), dim3(256), 0, 0, ob, Bs, S); }, by,
           "sweep store pattern SoA (rows 4 MB apart)");
    timeit([&] { hipLaunchKernelGGL(sweep_tiled, dim3(Bs / 2 / 256), dim3(256), 0, 0, ob, Bs, S); }, by,
           "sweep store pattern tiled (24 KB per wave per stage)");
    timeit([&] { hipLaunchKernelGGL(sweep_tilemajor, dim3(Bs / 2 / 256), dim3(256), 0, 0, ob, Bs, S); }, by,
           "sweep store pattern tile-major (480 KB per wave)");
    timeit([&] { hipLaunchKernelGGL(sweep_tiled64, dim3(Bs / 256), dim3(256), 0, 0, ob, Bs, S); }, by,
           "sweep store pattern tiled, 64-instance tiles, 8B/lane");
    CK(hipFree(ob));
    double *X, *U, *J;
    CK(hipMalloc(&X, (long)Bs * (S + 1) * 3 * 8));
    CK(hipMalloc(&U, (long)Bs * S * 2 * 8));
    CK(hipMalloc(&J, (long)Bs * S * 24 * 8));
    CK(hipMemset(X, 0, (long)Bs * (S + 1) * 3 * 8));
    CK(hipMemset(U, 0, (long)Bs * S * 2 * 8));
    const double byc = (double)Bs * ((S + 1) * 3 * 8 + S * 2 * 8 + S * 24 * 8);
    timeit([&] { hipLaunchKernelGGL(sweep_copy, dim3(Bs / 256), dim3(256), 0, 0, X, U, J, Bs, S); }, byc,
           "sweep traffic without arithmetic (compulsory bytes)");
    timeit([&] { hipLaunchKernelGGL(sweep_copy16<false>, dim3(Bs / 256), dim3(256), 0, 0, X, U, J, Bs, S); }, byc,
           "sweep traffic without arithmetic, 16-B record stores (field pairs)");
    timeit([&] { hipLaunchKernelGGL(sweep_copy16<true>, dim3(Bs / 256), dim3(256), 0, 0, X, U, J, Bs, S); }, byc,
           "sweep traffic without arithmetic, 16-B nontemporal record stores");
    timeit([&] { hipLaunchKernelGGL(sweep_copy16<true>, dim3(Bs / 64), dim3(64), 0, 0, X, U, J, Bs, S); }, byc,
           "sweep traffic without arithmetic, 16-B nt record stores, 64-thread blocks");
    const double byf = byc + (double)Bs * S * 3 * 8;  // x_{k+1} read twice
    timeit([&] { hipLaunchKernelGGL((sweep_flat<8, false>), dim3(Bs / 256 * S), dim3(256), 0, 0, X, U, J, Bs, S); }, byc,
           "flat (instance,stage) threads, 8-B stores (GB/s of compulsory bytes)");
    timeit([&] { hipLaunchKernelGGL((sweep_flat<8, true>), dim3(Bs / 256 * S), dim3(256), 0, 0, X, U, J, Bs, S); }, byc,
           "flat (instance,stage) threads, 8-B nt stores");
    timeit([&] { hipLaunchKernelGGL((sweep_flat<16, false>), dim3(Bs / 256 * S), dim3(256), 0, 0, X, U, J, Bs, S); }, byc,
           "flat (instance,stage) threads, 16-B stores");
    timeit([&] { hipLaunchKernelGGL((sweep_flat<16, true>), dim3(Bs / 256 * S), dim3(256), 0, 0, X, U, J, Bs, S); }, byc,
           "flat (instance,stage) threads, 16-B nt stores");
    timeit([&] { hipLaunchKernelGGL((sweep_flat<16, true>), dim3(Bs / 64 * S), dim3(64), 0, 0, X, U, J, Bs, S); }, byc,
           "flat (instance,stage) threads, 16-B nt stores, 64-thread blocks");
    (void)byf;
    CK(hipFree(X));
    CK(hipFree(U));
    CK(hipFree(J));
  }
  const long nm = nw / 4;
  timeit([&] { hipLaunchKernelGGL(mix, dim3(grid), dim3(block), 0, 0, a, o, nm); }, nm * 16.0 * (1 + 4.5),
         "read:write 1:4.5 16B/lane");
  return 0;
}
