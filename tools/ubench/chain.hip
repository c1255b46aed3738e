// Dependent-latency micro-benchmark (straight-line asm, no loop overhead): one wave.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench/chain.hip -o tools/ubench/chain
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)
#define R32(x) R16(x) R16(x)

__global__ void chain(unsigned long long* cyc, double* out, double a) {
  double x = a + threadIdx.x * 1e-3, y = 0.999, z = 1e-3;
  unsigned long long t0, t1, r0, r1;
  // 0: 32 dependent v_fma_f64
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile(R32("v_fma_f64 %0, %0, %1, %2\n\t") : "+v"(x) : "v"(y), "v"(z));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[0] = t1 - t0;
  // 1: 32 dependent v_add_f64
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile(R32("v_add_f64 %0, %0, %1\n\t") : "+v"(x) : "v"(z));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[1] = t1 - t0;
  // 2: 32 dependent v_fmac_f64_dpp row_newbcast (dependency through the accumulator)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_nop 1\n\t" R32("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t")
               : "+v"(x) : "v"(y), "v"(z));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[2] = t1 - t0;
  // 3: 32 dependent DPP through the broadcast operand (x = bcast(x) * y + acc)
  double acc = 0.0;
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile(R32("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t")
               : "+v"(x) : "v"(y));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[3] = t1 - t0;
  // 4: 32 dependent permlane32_swap pairs + add (pair_sum)
  double w = x;
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const long long b = __double_as_longlong(w);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    w = __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
    asm volatile("" : "+v"(w));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[4] = t1 - t0;
  // 5: 32 independent v_fma_f64 (issue rate)
  double q[8] = {x, x + 1, x + 2, x + 3, x + 4, x + 5, x + 6, x + 7};
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile(R4("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\t"
                  "v_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9\n\t")
               : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]), "+v"(q[4]), "+v"(q[5]), "+v"(q[6]), "+v"(q[7])
               : "v"(y), "v"(z));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[5] = t1 - t0;
  // 6: empty (timer overhead)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[6] = t1 - t0;
  // 7: clock ratio: s_memtime vs s_memrealtime (100 MHz) over a long dependent chain
  r0 = __builtin_amdgcn_s_memrealtime();
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 2000; ++i) asm volatile(R32("v_fma_f64 %0, %0, %1, %2\n\t") : "+v"(x) : "v"(y), "v"(z));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  r1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  cyc[7] = t1 - t0;
  cyc[8] = r1 - r0;
  // 9: 32 dependent LDS loads (pointer chasing through LDS)
  __shared__ int lds[64];
  lds[threadIdx.x] = (threadIdx.x + 1) & 63;
  __syncthreads();
  int idx = threadIdx.x;
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 32; ++i) { idx = lds[idx]; asm volatile("" : "+v"(idx)); }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[9] = t1 - t0;
  // 10: 32 dependent v_mov_b32_dpp row_ror (half_shift style, 32-bit)
  unsigned u = threadIdx.x;
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile(R32("s_nop 1\n\tv_mov_b32_dpp %0, %0 row_ror:10 row_mask:0xc bank_mask:0xf\n\t") : "+v"(u));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  cyc[10] = t1 - t0;
  double s = idx + u; for (int i = 0; i < 8; ++i) s += q[i];
  out[threadIdx.x] = x + w + s + acc;
}

int main() {
  unsigned long long* c; double* d;
  hipMalloc(&c, 16 * 8); hipMalloc(&d, 64 * 8);
  for (int rep = 0; rep < 3; ++rep) { hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, c, d, 1.0); hipDeviceSynchronize(); }
  unsigned long long h[16]; hipMemcpy(h, c, 16 * 8, hipMemcpyDeviceToHost);
  const char* nm[7] = {"v_fma_f64 dependent", "v_add_f64 dependent", "v_fmac_f64_dpp dep (acc)", "v_fmac_f64_dpp dep (bcast src)",
                       "pair_sum (permlane32 swap + add)", "v_fma_f64 8 independent chains (per instr)", "timer overhead"};
  for (int i = 0; i < 7; ++i) printf("%-44s %7.1f cycles %s\n", nm[i], (double)(h[i] - (i < 6 ? h[6] : 0)) / (i == 6 ? 1 : 32),
                                      i == 6 ? "(total)" : "per op");
  printf("%-44s %7.1f cycles per op\n", "LDS load dependent (ds_read_b32)", (double)(h[9] - h[6]) / 32);
  printf("%-44s %7.1f cycles per op\n", "v_mov_b32_dpp row_ror dep (+s_nop 1)", (double)(h[10] - h[6]) / 32);
  printf("memtime/memrealtime ratio: %.2f (memtime MHz if realtime is 100 MHz: %.0f)\n", (double)h[7] / h[8], 100.0 * h[7] / h[8]);
  printf("long chain: %.2f memtime cycles per dependent fma\n", (double)h[7] / (2000.0 * 32));
  return 0;
}
