// Latency micro-benchmarks for the sweep chain's building blocks (one wave).
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  return __longlong_as_double(__builtin_amdgcn_mov_dpp(__double_as_longlong(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ double pair_sum(double v) {
  const long long b = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

__global__ void lat(double* out, unsigned long long* cyc, int n, double a) {
  double x = a + threadIdx.x * 1e-3;
  unsigned long long t0, t1;
  __shared__ double buf[64];
  // 0: dependent fma chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) { x = fma(x, 0.999, 1e-3); asm volatile("" : "+v"(x)); }
  t1 = __builtin_amdgcn_s_memtime(); cyc[0] = t1 - t0;
  // 1: dpp newbcast + fma
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) { x = fma(dpp64<0x153>(x), 0.999, 1e-3); asm volatile("" : "+v"(x)); }
  t1 = __builtin_amdgcn_s_memtime(); cyc[1] = t1 - t0;
  // 2: pair_sum (permlane32 swap) + scale
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) { x = pair_sum(x) * 0.5; asm volatile("" : "+v"(x)); }
  t1 = __builtin_amdgcn_s_memtime(); cyc[2] = t1 - t0;
  // 3: LDS write -> read round trip in one wave
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    buf[threadIdx.x] = x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    x = buf[(threadIdx.x + 1) & 63] * 0.999;
    asm volatile("" : "+v"(x));
  }
  t1 = __builtin_amdgcn_s_memtime(); cyc[3] = t1 - t0;
  // 4: quad_perm (32-bit pairs) + add
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) { x = x + dpp64<0xB1>(x) * 0.5; asm volatile("" : "+v"(x)); }
  t1 = __builtin_amdgcn_s_memtime(); cyc[4] = t1 - t0;
  // 5: independent fma throughput (4 chains)
  double y0 = x, y1 = x + 1, y2 = x + 2, y3 = x + 3;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    y0 = fma(y0, 0.999, 1e-3); y1 = fma(y1, 0.999, 1e-3); y2 = fma(y2, 0.999, 1e-3); y3 = fma(y3, 0.999, 1e-3);
    asm volatile("" : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
  }
  t1 = __builtin_amdgcn_s_memtime(); cyc[5] = t1 - t0;
  // 6: 12 independent dpp newbcast (issue rate)
  double z[12];
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    z[0] = dpp64<0x150>(x); z[1] = dpp64<0x151>(x); z[2] = dpp64<0x152>(x); z[3] = dpp64<0x153>(x);
    z[4] = dpp64<0x154>(x); z[5] = dpp64<0x155>(x); z[6] = dpp64<0x156>(x); z[7] = dpp64<0x157>(x);
    z[8] = dpp64<0x158>(x); z[9] = dpp64<0x159>(x); z[10] = dpp64<0x15A>(x); z[11] = dpp64<0x15B>(x);
    asm volatile("" : "+v"(z[0]), "+v"(z[1]), "+v"(z[2]), "+v"(z[3]), "+v"(z[4]), "+v"(z[5]), "+v"(z[6]),
                 "+v"(z[7]), "+v"(z[8]), "+v"(z[9]), "+v"(z[10]), "+v"(z[11]));
  }
  t1 = __builtin_amdgcn_s_memtime(); cyc[6] = t1 - t0;
  // 7: s_barrier alone (4 waves)
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) { __syncthreads(); }
  t1 = __builtin_amdgcn_s_memtime(); cyc[7] = t1 - t0;
  double zz = 0; for (int i = 0; i < 12; ++i) zz += z[i];
  out[threadIdx.x] = x + y0 + y1 + y2 + y3 + zz;
}

int main() {
  double* d; unsigned long long* c; hipMalloc(&d, 256 * 8); hipMalloc(&c, 16 * 8);
  const int n = 1000;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(256), 0, 0, d, c, n, 1.0);
    hipDeviceSynchronize();
  }
  unsigned long long h[16]; hipMemcpy(h, c, 16 * 8, hipMemcpyDeviceToHost);
  const char* nm[8] = {"fma f64 dep", "dpp64 bcast+fma dep", "permlane32 pair_sum+mul dep", "lds write->read dep",
                       "quad_perm dpp(2x32)+fma dep", "fma f64 4 indep chains (per iter)", "12 dpp64 indep (per iter)",
                       "s_barrier 4 waves"};
  for (int i = 0; i < 8; ++i) printf("%-36s %8.1f cycles/iter\n", nm[i], (double)h[i] / n);
  return 0;
}
