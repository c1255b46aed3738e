// Does the LDS serve an exec-masked read faster?  The sweeps' reads, one round = 6 reads
// then a wait, with every lane active (the engine's form: duplicate lanes re-read data
// other lanes read) against the same reads with only the lanes that need the data active:
//   col  outward columns, 6 ds_read2_b64: lane l reads doubles (l & 15) % 12 (+ 12 i) of its
//        chain's block (rows 0/1 two blocks, rows 2/3 repeat rows 0/1)
//        masks: all 64 lanes | rows 0/1 with s < 12 (24 lanes) | rows 0/1 (32 lanes)
//   row  inward rows, 6 ds_read_b128: lane l reads 96-B row (l & 15) % 12 of its row's block
//        (four blocks: rows 0..3)
//        masks: all 64 lanes | s < 12 in every row (48 lanes)
// s_memtime ticks per round, 1 / 4 / 8 waves per workgroup (one workgroup per CU).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ldsx tools/ubench/lds_exec.hip && /tmp/ldsx
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int V>
__global__ void kern(double* out, long long* cyc, int reps, unsigned long long mask) {
  __shared__ double lds[12288];
  for (int i = threadIdx.x; i < 12288; i += blockDim.x) lds[i] = i;
  __syncthreads();
  const int l = threadIdx.x & 63, s = l & 15, row = l >> 4;
  const int w = threadIdx.x >> 6;
  // outward: block of chain (row & 1), column s % 12; RS = 12 doubles; blocks 1280 doubles apart
  const unsigned acol = 8u * (unsigned)(w * 1500 + (row & 1) * 1280 + s % 12);
  // inward: 96-B rows, row s % 12 of block row
  const unsigned arow = 8u * (unsigned)(w * 1500 + row * 160 + 12 * (s % 12));
  d2 v0 = {0, 0}, v1 = v0, v2 = v0, v3 = v0, v4 = v0, v5 = v0;
  unsigned long long sv;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    if constexpr (V == 0) {
      asm volatile(
          "s_mov_b64 %6, exec\n s_mov_b64 exec, %8\n"
          "ds_read2_b64 %0, %7 offset1:12\n ds_read2_b64 %1, %7 offset0:24 offset1:36\n"
          "ds_read2_b64 %2, %7 offset0:48 offset1:60\n ds_read2_b64 %3, %7 offset0:72 offset1:84\n"
          "ds_read2_b64 %4, %7 offset0:96 offset1:108\n ds_read2_b64 %5, %7 offset0:120 offset1:132\n"
          "s_mov_b64 exec, %6\n s_waitcnt lgkmcnt(0)\n"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "=&s"(sv)
          : "v"(acol), "s"(mask)
          : "memory");
    } else {
      asm volatile(
          "s_mov_b64 %6, exec\n s_mov_b64 exec, %8\n"
          "ds_read_b128 %0, %7\n ds_read_b128 %1, %7 offset:16\n ds_read_b128 %2, %7 offset:32\n"
          "ds_read_b128 %3, %7 offset:48\n ds_read_b128 %4, %7 offset:64\n ds_read_b128 %5, %7 offset:80\n"
          "s_mov_b64 exec, %6\n s_waitcnt lgkmcnt(0)\n"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "=&s"(sv)
          : "v"(arow), "s"(mask)
          : "memory");
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = v0.x + v1.x + v2.x + v3.x + v4.x + v5.x + v0.y + v5.y;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(const char* name, int waves, unsigned long long mask) {
  const int reps = 2000, blocks = 256;
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, sizeof(double) * blocks * 64 * waves);
  (void)hipMalloc(&cyc, sizeof(long long) * blocks);
  kern<V><<<blocks, 64 * waves>>>(out, cyc, reps, mask);
  kern<V><<<blocks, 64 * waves>>>(out, cyc, reps, mask);
  long long h[256];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  printf("%-44s waves %d: %7.2f ticks per round of 6 reads\n", name, waves, m / reps);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  const unsigned long long all = ~0ull, s12 = 0x0FFF0FFF0FFF0FFFull, half0 = 0xFFFFFFFFull,
                           half0s12 = 0x0FFF0FFFull;
  for (int w : {1, 4, 8}) {
    run<0>("col ds_read2_b64, all 64 lanes", w, all);
    run<0>("col ds_read2_b64, rows 0/1 s<12 (24 lanes)", w, half0s12);
    run<0>("col ds_read2_b64, rows 0/1 (32 lanes)", w, half0);
    run<1>("row ds_read_b128, all 64 lanes", w, all);
    run<1>("row ds_read_b128, s<12 (48 lanes)", w, s12);
  }
  return 0;
}
