// Microbenchmark: issue cost of the LDS / cross-lane instructions of the sweeps,
// one wave per SIMD.  Ticks of s_memtime per instruction.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lds tools/ubench_lds.hip && tools/ubench_lds
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R2(x) x x
#define R6(x) x x x x x x

template <int V>
__global__ void kern(double* out, long long* cyc, int reps) {
  __shared__ double lds[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = i;
  __syncthreads();
  const unsigned a = (unsigned)(threadIdx.x & 15) * 96u + (threadIdx.x >> 4) * 2304u;  // sweep-row pattern
  double v0 = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0, v5 = 0, acc = 1.0, g = 0.5;
  unsigned u0 = threadIdx.x, u1 = 3;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    if constexpr (V == 0) {  // 6 x ds_read_b128, waited once (a sweep row)
      asm volatile("ds_read_b128 %0, %6\n ds_read_b128 %1, %6 offset:16\n ds_read_b128 %2, %6 offset:32\n"
                   "ds_read_b128 %3, %6 offset:48\n ds_read_b128 %4, %6 offset:64\n ds_read_b128 %5, %6 offset:80\n"
                   "s_waitcnt lgkmcnt(0)\n"
                   : "=v"(*(double2*)&v0), "=v"(*(double2*)&v1), "=v"(*(double2*)&v2), "=v"(*(double2*)&v3),
                     "=v"(*(double2*)&v4), "=v"(*(double2*)&v5) : "v"(a) : "memory");
    } else if constexpr (V == 1) {  // 6 x ds_read_b128 issued, waited one round later (prefetch), + 12 fma
      asm volatile("ds_read_b128 %0, %6\n ds_read_b128 %1, %6 offset:16\n ds_read_b128 %2, %6 offset:32\n"
                   "ds_read_b128 %3, %6 offset:48\n ds_read_b128 %4, %6 offset:64\n ds_read_b128 %5, %6 offset:80\n"
                   : "=v"(*(double2*)&v0), "=v"(*(double2*)&v1), "=v"(*(double2*)&v2), "=v"(*(double2*)&v3),
                     "=v"(*(double2*)&v4), "=v"(*(double2*)&v5) : "v"(a) : "memory");
      asm volatile(R6("v_fmac_f64 %0, %1, %1\n v_fmac_f64 %0, %1, %1\n") : "+v"(acc) : "v"(g));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if constexpr (V == 2) {  // 12 fma alone (reference for V == 1)
      asm volatile(R6("v_fmac_f64 %0, %1, %1\n v_fmac_f64 %0, %1, %1\n") : "+v"(acc) : "v"(g));
    } else if constexpr (V == 3) {  // 6 x ds_read2_b64 (column pairs), waited once
      asm volatile("ds_read2_b64 %0, %6 offset1:12\n ds_read2_b64 %1, %6 offset0:24 offset1:36\n"
                   "ds_read2_b64 %2, %6 offset0:48 offset1:60\n ds_read2_b64 %3, %6 offset0:72 offset1:84\n"
                   "ds_read2_b64 %4, %6 offset0:96 offset1:108\n ds_read2_b64 %5, %6 offset0:120 offset1:132\n"
                   "s_waitcnt lgkmcnt(0)\n"
                   : "=v"(*(double2*)&v0), "=v"(*(double2*)&v1), "=v"(*(double2*)&v2), "=v"(*(double2*)&v3),
                     "=v"(*(double2*)&v4), "=v"(*(double2*)&v5) : "v"(a) : "memory");
    } else if constexpr (V == 4) {  // 6 x ds_write_b64
      asm volatile(R6("ds_write_b64 %0, %1 offset:8192\n") "s_waitcnt lgkmcnt(0)\n" : : "v"(a), "v"(acc) : "memory");
    } else if constexpr (V == 5) {  // 6 x v_mov_b64_dpp
      asm volatile(R6("v_mov_b64_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n") : "=v"(v0) : "v"(acc));
    } else if constexpr (V == 6) {  // 6 x v_cndmask_b32
      asm volatile(R6("v_cndmask_b32 %0, %0, %1, vcc\n") : "+v"(u0) : "v"(u1));
    } else if constexpr (V == 7) {  // 6 x v_permlane16_swap_b32
      asm volatile(R6("v_permlane16_swap_b32 %0, %1\n") : "+v"(u0), "+v"(u1));
    } else if constexpr (V == 8) {  // 6 x v_add_u32
      asm volatile(R6("v_add_u32 %0, %0, %1\n") : "+v"(u0) : "v"(u1));
    } else if constexpr (V == 9) {  // 6 x ds_read_b64, waited once
      asm volatile("ds_read_b64 %0, %6\n ds_read_b64 %1, %6 offset:8\n ds_read_b64 %2, %6 offset:16\n"
                   "ds_read_b64 %3, %6 offset:24\n ds_read_b64 %4, %6 offset:32\n ds_read_b64 %5, %6 offset:40\n"
                   "s_waitcnt lgkmcnt(0)\n"
                   : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5) : "v"(a) : "memory");
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + acc + u0 + u1;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(const char* name, int waves, int per) {
  const int reps = 2000, blocks = 256;
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, sizeof(double) * blocks * 64 * waves);
  (void)hipMalloc(&cyc, sizeof(long long) * blocks);
  kern<V><<<blocks, 64 * waves>>>(out, cyc, reps);
  kern<V><<<blocks, 64 * waves>>>(out, cyc, reps);
  long long h[256];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  printf("%-58s waves %d: %7.2f ticks per round, %6.2f per instruction\n", name, waves, m / reps, m / (reps * per));
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  for (int w : {1, 4}) {
    run<0>("6 ds_read_b128 (sweep-row pattern) + wait", w, 6);
    run<1>("6 ds_read_b128 + 12 fma, then wait", w, 18);
    run<2>("12 fma", w, 12);
    run<3>("6 ds_read2_b64 (columns) + wait", w, 6);
    run<9>("6 ds_read_b64 + wait", w, 6);
    run<4>("6 ds_write_b64 + wait", w, 6);
    run<5>("6 v_mov_b64_dpp", w, 6);
    run<6>("6 v_cndmask_b32", w, 6);
    run<7>("6 v_permlane16_swap_b32", w, 6);
    run<8>("6 v_add_u32", w, 6);
  }
  return 0;
}
