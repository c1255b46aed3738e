// Microbenchmark: issue cost of the FP64 instructions the sweeps are built from,
// one wave per SIMD (the sweep wave's situation).  Cycles from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_fma tools/ubench_fma.hip && /tmp/ubench_fma
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R4(x) x x x x
#define R12(x) R4(x) R4(x) R4(x)

template <int V>
__global__ void kern(double* out, long long* cyc, int reps) {
  double acc = threadIdx.x * 1e-3, acc2 = 1.0 + threadIdx.x, src = 0.5 + threadIdx.x * 1e-6, g = 0.999;
  double a3 = 2.0, a4 = 3.0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    if constexpr (V == 0) {  // dependent v_fmac_f64_dpp chain (row broadcast)
      asm volatile(R12("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n") : "+v"(acc) : "v"(src), "v"(g));
    } else if constexpr (V == 1) {  // dependent plain v_fmac_f64 chain
      asm volatile(R12("v_fmac_f64 %0, %1, %2\n") : "+v"(acc) : "v"(src), "v"(g));
    } else if constexpr (V == 2) {  // two independent dpp chains interleaved (12 instructions)
      asm volatile(R4("v_fmac_f64_dpp %0, %2, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                      "v_fmac_f64_dpp %1, %2, %3 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                      "v_fmac_f64_dpp %0, %2, %3 row_newbcast:7 row_mask:0xf bank_mask:0xf\n")
                   : "+v"(acc), "+v"(acc2) : "v"(src), "v"(g));
    } else if constexpr (V == 3) {  // four independent plain chains (12 instructions)
      asm volatile(R4("v_fmac_f64 %0, %4, %5\n v_fmac_f64 %1, %4, %5\n v_fmac_f64 %2, %4, %5\n")
                   : "+v"(acc), "+v"(acc2), "+v"(a3), "+v"(a4) : "v"(src), "v"(g));
    } else if constexpr (V == 4) {  // dependent v_add_f64 chain
      asm volatile(R12("v_add_f64 %0, %0, %1\n") : "+v"(acc) : "v"(g));
    } else if constexpr (V == 5) {  // permlane32 swap pairs (2 x b32 each), 6 pairs
      unsigned lo = (unsigned)threadIdx.x, hi = lo * 3u;
      asm volatile(R4("v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %1, %0\n v_permlane32_swap_b32 %0, %1\n")
                   : "+v"(lo), "+v"(hi));
      acc += lo + hi;
    } else if constexpr (V == 6) {  // dependent v_fma_f64 (3 operands, no dpp)
      asm volatile(R12("v_fma_f64 %0, %1, %2, %0\n") : "+v"(acc) : "v"(src), "v"(g));
    } else if constexpr (V == 7) {  // dependent v_mul_f64 chain
      asm volatile(R12("v_mul_f64 %0, %0, %1\n") : "+v"(acc) : "v"(g));
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc + acc2 + a3 + a4;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(const char* name, int waves_per_block) {
  const int reps = 2000, blocks = 256;
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * 64 * waves_per_block);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  kern<V><<<blocks, 64 * waves_per_block>>>(out, cyc, reps);  // warm-up
  kern<V><<<blocks, 64 * waves_per_block>>>(out, cyc, reps);
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  printf("%-44s waves/block %d: %.2f cycles per instruction\n", name, waves_per_block, m / (reps * 12.0));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w : {1, 4}) {
    run<0>("dependent v_fmac_f64_dpp row_newbcast", w);
    run<1>("dependent v_fmac_f64", w);
    run<6>("dependent v_fma_f64", w);
    run<2>("two interleaved v_fmac_f64_dpp chains", w);
    run<3>("four interleaved v_fmac_f64 chains", w);
    run<4>("dependent v_add_f64", w);
    run<7>("dependent v_mul_f64", w);
    run<5>("v_permlane32_swap_b32", w);
  }
  return 0;
}
