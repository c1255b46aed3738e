// Issue-rate micro-benchmark: 32 independent instructions of one kind, one wave.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench/issue.hip -o tools/ubench/issue
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R4(x) x x x x
#define R8(x) R4(x) R4(x)
#define T0 asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); t0 = __builtin_amdgcn_s_memtime(); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#define T1(i) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(0)" ::: "memory"); t1 = __builtin_amdgcn_s_memtime(); cyc[i] = t1 - t0;

__global__ void issue(unsigned long long* cyc, double* out, double a) {
  __shared__ double lds[64 * 16];
  for (int i = threadIdx.x; i < 64 * 16; i += 64) lds[i] = i;
  __syncthreads();
  double x0 = a + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  double y = 0.5, z = 1e-3;
  unsigned long long t0, t1;
  unsigned addr = threadIdx.x * 8 * 13;
  // 0: empty
  T0 T1(0)
  // 1: 32 independent v_fma_f64 (8 chains x 4)
  T0 asm volatile(R4("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\t"
                     "v_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9\n\t")
                  : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y), "v"(z)); T1(1)
  // 2: 32 independent v_fmac_f64_dpp row_newbcast (8 accumulators)
  T0 asm volatile("s_nop 1\n\t" R4("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t")
                  : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y), "v"(z)); T1(2)
  // 3: 32 independent v_fmac_f64 (no dpp)
  T0 asm volatile(R4("v_fmac_f64 %0, %8, %9\n\tv_fmac_f64 %1, %8, %9\n\tv_fmac_f64 %2, %8, %9\n\tv_fmac_f64 %3, %8, %9\n\t"
                     "v_fmac_f64 %4, %8, %9\n\tv_fmac_f64 %5, %8, %9\n\tv_fmac_f64 %6, %8, %9\n\tv_fmac_f64 %7, %8, %9\n\t")
                  : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y), "v"(z)); T1(3)
  // 4: 32 ds_read2_b64 (16 B per lane, stride 13 doubles between lanes)
  double r[8];
  T0 asm volatile(R4("ds_read2_b64 %0, %4 offset1:1\n\tds_read2_b64 %1, %4 offset0:2 offset1:3\n\t"
                     "ds_read2_b64 %2, %4 offset0:4 offset1:5\n\tds_read2_b64 %3, %4 offset0:6 offset1:7\n\t")
                     R4("ds_read2_b64 %0, %4 offset1:1\n\tds_read2_b64 %1, %4 offset0:2 offset1:3\n\t"
                     "ds_read2_b64 %2, %4 offset0:4 offset1:5\n\tds_read2_b64 %3, %4 offset0:6 offset1:7\n\t")
                  : "=v"(*(double2*)&r[0]), "=v"(*(double2*)&r[2]), "=v"(*(double2*)&r[4]), "=v"(*(double2*)&r[6]) : "v"(addr)); T1(4)
  // 5: 32 ds_read_b64 broadcast (all lanes same address)
  unsigned a0 = 0;
  T0 asm volatile(R8("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:8\n\tds_read_b64 %2, %4 offset:16\n\tds_read_b64 %3, %4 offset:24\n\t")
                  : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]) : "v"(a0)); T1(5)
  // 6: 32 v_mov_b64_dpp row_newbcast
  T0 asm volatile("s_nop 1\n\t" R4("v_mov_b64_dpp %0, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b64_dpp %1, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_mov_b64_dpp %3, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %4, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\tv_mov_b64_dpp %5, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %6, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\tv_mov_b64_dpp %7, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t")
                  : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3), "=v"(x4), "=v"(x5), "=v"(x6), "=v"(x7) : "v"(y)); T1(6)
  // 7: 32 v_cndmask_b32 + v_add_u32 pairs (integer/select issue)
  unsigned u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3;
  T0 asm volatile(R8("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4\n\t")
                  : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(addr)); T1(7)
  // 8: 16 v_permlane32_swap pairs (32 instructions)
  unsigned p0 = u0, p1 = u1, p2 = u2, p3 = u3;
  T0 asm volatile(R8("v_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3\n\t") R8("v_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3\n\t")
                  : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)); T1(8)
  // 9: 32 ds_write_b64 (stride 13 doubles)
  T0 asm volatile(R8("ds_write_b64 %0, %1\n\tds_write_b64 %0, %1 offset:8\n\tds_write_b64 %0, %1 offset:16\n\tds_write_b64 %0, %1 offset:24\n\t")
                  : : "v"(addr), "v"(y) : "memory"); T1(9)
  // 10: 32 v_add_f64 independent
  T0 asm volatile(R4("v_add_f64 %0, %0, %8\n\tv_add_f64 %1, %1, %8\n\tv_add_f64 %2, %2, %8\n\tv_add_f64 %3, %3, %8\n\t"
                     "v_add_f64 %4, %4, %8\n\tv_add_f64 %5, %5, %8\n\tv_add_f64 %6, %6, %8\n\tv_add_f64 %7, %7, %8\n\t")
                  : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(z)); T1(10)
  // 11: 32 ds_read_b64 with lane stride 13 doubles (conflict-free pattern)
  T0 asm volatile(R8("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:8\n\tds_read_b64 %2, %4 offset:16\n\tds_read_b64 %3, %4 offset:24\n\t")
                  : "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]) : "v"(addr)); T1(11)
  // 12: 32 ds_read_b64 with lane stride 12 doubles (the unpadded sweep pattern)
  unsigned addr12 = threadIdx.x * 8 * 12;
  T0 asm volatile(R8("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:8\n\tds_read_b64 %2, %4 offset:16\n\tds_read_b64 %3, %4 offset:24\n\t")
                  : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]) : "v"(addr12)); T1(12)
  // 13: 32 ds_read2_b64 offsets (i, i+6), lane stride 13 doubles
  T0 asm volatile(R8("ds_read2_b64 %0, %4 offset1:6\n\tds_read2_b64 %1, %4 offset0:1 offset1:7\n\t"
                     "ds_read2_b64 %2, %4 offset0:2 offset1:8\n\tds_read2_b64 %3, %4 offset0:3 offset1:9\n\t")
                  : "=v"(*(double2*)&r[0]), "=v"(*(double2*)&r[2]), "=v"(*(double2*)&r[4]), "=v"(*(double2*)&r[6]) : "v"(addr)); T1(13)
  // 14: 32 ds_read2_b64 offsets (i, i+1), lane stride 12 doubles
  T0 asm volatile(R8("ds_read2_b64 %0, %4 offset1:1\n\tds_read2_b64 %1, %4 offset0:2 offset1:3\n\t"
                     "ds_read2_b64 %2, %4 offset0:4 offset1:5\n\tds_read2_b64 %3, %4 offset0:6 offset1:7\n\t")
                  : "=v"(*(double2*)&r[0]), "=v"(*(double2*)&r[2]), "=v"(*(double2*)&r[4]), "=v"(*(double2*)&r[6]) : "v"(addr12)); T1(14)
  // 15: 32 ds_read_b128, lane stride 12 doubles (16-B aligned)
  T0 asm volatile(R8("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\t")
                  : "=v"(*(double2*)&r[0]), "=v"(*(double2*)&r[2]), "=v"(*(double2*)&r[4]), "=v"(*(double2*)&r[6]) : "v"(addr12)); T1(15)
  // 16: 32 ds_read2_b64 offsets (i, i+13), lane stride 1 double (column reads of a 13-stride matrix)
  unsigned addr1 = threadIdx.x * 8;
  T0 asm volatile(R8("ds_read2_b64 %0, %4 offset1:13\n\tds_read2_b64 %1, %4 offset0:26 offset1:39\n\t"
                     "ds_read2_b64 %2, %4 offset0:52 offset1:65\n\tds_read2_b64 %3, %4 offset0:78 offset1:91\n\t")
                  : "=v"(*(double2*)&r[0]), "=v"(*(double2*)&r[2]), "=v"(*(double2*)&r[4]), "=v"(*(double2*)&r[6]) : "v"(addr1)); T1(16)
  double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + u0 + u1 + u2 + u3 + p0 + p1 + p2 + p3;
  for (int i = 0; i < 8; ++i) s += r[i];
  out[threadIdx.x] = s;
}

int main() {
  unsigned long long* c; double* d;
  (void)hipMalloc(&c, 32 * 8); (void)hipMalloc(&d, 64 * 8);
  for (int rep = 0; rep < 3; ++rep) { hipLaunchKernelGGL(issue, dim3(1), dim3(64), 0, 0, c, d, 1.0); (void)hipDeviceSynchronize(); }
  unsigned long long h[32]; (void)hipMemcpy(h, c, 32 * 8, hipMemcpyDeviceToHost);
  const char* nm[17] = {"empty", "v_fma_f64", "v_fmac_f64_dpp", "v_fmac_f64", "ds_read2_b64 (stride 13)", "ds_read_b64 broadcast",
                        "v_mov_b64_dpp", "v_add_u32", "v_permlane32_swap", "ds_write_b64 (stride 13)", "v_add_f64",
                        "ds_read_b64 (stride 13)", "ds_read_b64 (stride 12)",
                        "ds_read2_b64 (i,i+6) stride 13", "ds_read2_b64 (i,i+1) stride 12", "ds_read_b128 stride 12",
                        "ds_read2_b64 (i,i+13) stride 1"};
  printf("timer overhead %llu cycles\n", h[0]);
  for (int i = 1; i < 17; ++i) printf("%-28s %6.2f cycles per instruction (32 independent, incl. drain)\n", nm[i], (double)(h[i] - h[0]) / 32);
  return 0;
}
