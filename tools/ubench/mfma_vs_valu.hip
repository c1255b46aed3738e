// The factorisation's 12 x 12 products on VALU (the engine's form) against
// v_mfma_f64_16x16x4f64, one wave, s_memtime cycles (the unit
// of tools/factime.py and the stamps):
//   valu     four 12x12x12 products at once, one per 16-lane row, row ph of A in lane ph
//            (12 VGPRs), B's rows broadcast by v_fmac_f64_dpp row_newbcast -- 144 chained
//            instructions, the form of schur_cols / the Gauss-Jordan updates
//   mfma     one 12x12x12 product (padded to 16) as four dependent 16x16x4 MFMAs, operands
//            already in the MFMA lane maps (tools/ubench/mfma_f64_layout.hip)
//   mfma4    four independent products (four accumulators): the MFMA pipe's issue rate
//   mfma+cv  one product including the conversions from / to the row-per-lane layout
//            the factorisation keeps (A and B through LDS, D back to rows of 12)
//   mfma_dep 16 dependent MFMAs (latency per MFMA)
// Every product's result is checked against a host reference.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mvv tools/ubench/mfma_vs_valu.hip && /tmp/mvv
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

#define FENCE asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#define TIC FENCE; t0 = __builtin_amdgcn_s_memtime(); FENCE;
#define TOC(i) FENCE; cyc[i] = __builtin_amdgcn_s_memtime() - t0;

// one column of the VALU product: a = sum_k A[ph][k] (lane ph) * B[k][c] (lane k)
#define BC(J, K) "v_fmac_f64_dpp %0, %1, %" #K " row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ double col12(const double (&a)[12], double bc) {
  // acc = sum_k a[k] * bc(lane k): the broadcast operand is B's column c held per lane
  double acc = 0.0;
  asm volatile("s_nop 1\n\t" BC(0, 2) BC(1, 3) BC(2, 4) BC(3, 5) BC(4, 6) BC(5, 7) BC(6, 8) BC(7, 9) BC(8, 10)
                   BC(9, 11) BC(10, 12) BC(11, 13)
               : "+v"(acc)
               : "v"(bc), "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
                 "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]));
  return acc;
}

__global__ void bench(const double* A, const double* B, double* out, unsigned long long* cyc) {
  __shared__ double lds[3 * 256];
  const int l = threadIdx.x, ph = l & 15;
  unsigned long long t0;
  // ---- VALU: row ph of A (zero beyond 12), B's row ph in lane ph
  double a[12], b[12];
  for (int k = 0; k < 12; ++k) { a[k] = ph < 12 ? A[12 * ph + k] : 0.0; b[k] = ph < 12 ? B[12 * ph + k] : 0.0; }
  double o[12];
  TIC
#pragma unroll
  for (int c = 0; c < 12; ++c) o[c] = col12(a, b[c]);
  TOC(0)
  for (int c = 0; c < 12; ++c) out[64 * c + l] = o[c];
  // ---- MFMA, operands in the MFMA maps: A[i][4s + k] at lane i + 16 k, B[4s + k][j] at lane j + 16 k
  const int i = l & 15, kk = l >> 4;
  double am[4], bm[4];
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + kk;
    am[s] = (i < 12 && k < 12) ? A[12 * i + k] : 0.0;
    bm[s] = (k < 12 && i < 12) ? B[12 * k + i] : 0.0;
  }
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  TIC
  asm volatile("" : "+v"(am[0]), "+v"(am[1]), "+v"(am[2]), "+v"(am[3]), "+v"(bm[0]), "+v"(bm[1]), "+v"(bm[2]), "+v"(bm[3]));
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(am[s], bm[s], acc, 0, 0, 0);
  asm volatile("" : "+v"(acc));
  TOC(1)
  for (int r = 0; r < 4; ++r) out[768 + 64 * r + l] = acc[r];
  // ---- four independent products (issue rate)
  d4 q0 = {0, 0, 0, 0}, q1 = q0, q2 = q0, q3 = q0;
  double a1[4], a2[4], a3[4];  // distinct operands (no common subexpressions)
  for (int s = 0; s < 4; ++s) { a1[s] = 2.0 * am[s]; a2[s] = 3.0 * am[s]; a3[s] = 4.0 * am[s]; }
  asm volatile("" : "+v"(a1[0]), "+v"(a1[1]), "+v"(a1[2]), "+v"(a1[3]), "+v"(a2[0]), "+v"(a2[1]), "+v"(a2[2]),
               "+v"(a2[3]), "+v"(a3[0]), "+v"(a3[1]), "+v"(a3[2]), "+v"(a3[3]));
  TIC
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    q0 = __builtin_amdgcn_mfma_f64_16x16x4f64(am[s], bm[s], q0, 0, 0, 0);
    q1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s], bm[s], q1, 0, 0, 0);
    q2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s], bm[s], q2, 0, 0, 0);
    q3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a3[s], bm[s], q3, 0, 0, 0);
  }
  asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3));
  TOC(2)
  for (int r = 0; r < 4; ++r) out[1024 + 64 * r + l] = q0[r] + q1[r] + q2[r] - q3[r];  // (1 + 2 + 3 - 4) P = 2 P
  // ---- MFMA with the conversions: rows of 12 (lane ph) -> LDS -> MFMA maps -> D -> LDS -> rows
  double oc[12];
  TIC
  if (l < 16)
    for (int k = 0; k < 12; ++k) { lds[16 * ph + k] = a[k]; lds[256 + 16 * ph + k] = b[k]; }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  double ac[4], bcv[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + kk;
    ac[s] = k < 12 ? lds[16 * i + k] : 0.0;
    bcv[s] = k < 12 ? lds[256 + 16 * k + i] : 0.0;
  }
  d4 dc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s) dc = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[s], bcv[s], dc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) lds[512 + 16 * (kk + 4 * r) + i] = dc[r];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int c = 0; c < 12; ++c) oc[c] = lds[512 + 16 * ph + c];
  TOC(3)
  for (int c = 0; c < 12; ++c) out[1280 + 64 * c + l] = oc[c];
  // ---- 16 dependent MFMAs
  d4 dd = acc;
  TIC
#pragma unroll
  for (int r = 0; r < 16; ++r) dd = __builtin_amdgcn_mfma_f64_16x16x4f64(am[r & 3], bm[r & 3], dd, 0, 0, 0);
  asm volatile("" : "+v"(dd));
  TOC(4)
  out[2048 + l] = dd[0] + dd[1] + dd[2] + dd[3];
  // ---- 144 dependent v_fmac_f64 (the same count as the VALU product, one chain)
  double ch = a[0];
  TIC
#pragma unroll
  for (int r = 0; r < 12; ++r) ch = col12(a, ch);
  TOC(5)
  out[2112 + l] = ch;
  // ---- the timing brackets alone
  TIC
  TOC(6)
}

int main() {
  double hA[144], hB[144], ref[144];
  for (int r = 0; r < 12; ++r)
    for (int c = 0; c < 12; ++c) {
      hA[12 * r + c] = ((r * 7 + c * 3) % 11 - 5) * 0.25;
      hB[12 * r + c] = ((r * 5 + c * c) % 13 - 6) * 0.5;
    }
  for (int r = 0; r < 12; ++r)
    for (int c = 0; c < 12; ++c) {
      double s = 0;
      for (int k = 0; k < 12; ++k) s += hA[12 * r + k] * hB[12 * k + c];
      ref[12 * r + c] = s;
    }
  double *dA, *dB, *dO;
  unsigned long long* dC;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dO, 4096 * 8); hipMalloc(&dC, 16 * 8);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  unsigned long long best[7];
  for (int i = 0; i < 7; ++i) best[i] = ~0ull;
  static double hO[4096];
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL(bench, dim3(1), dim3(64), 0, 0, dA, dB, dO, dC);
    unsigned long long c[16];
    hipMemcpy(c, dC, sizeof c, hipMemcpyDeviceToHost);
    for (int i = 0; i < 7; ++i) best[i] = c[i] < best[i] ? c[i] : best[i];
  }
  hipMemcpy(hO, dO, sizeof hO, hipMemcpyDeviceToHost);
  int bad_v = 0, bad_m = 0, bad_c = 0, bad_4 = 0;
  for (int r = 0; r < 12; ++r)
    for (int c = 0; c < 12; ++c) {
      const double e = ref[12 * r + c];
      bad_v += fabs(hO[64 * c + r] - e) > 1e-12;                      // VALU: column c in out[64 c + lane r]
      bad_m += fabs(hO[768 + 64 * (r >> 2) + c + 16 * (r & 3)] - e) > 1e-12;  // D row r: reg r>>2, lane c + 16 (r&3)
      bad_c += fabs(hO[1280 + 64 * c + r] - e) > 1e-12;
      bad_4 += fabs(hO[1024 + 64 * (r >> 2) + c + 16 * (r & 3)] - 2.0 * e) > 1e-11;
    }
  printf("check: valu %d, mfma %d, mfma4 %d, mfma+conversion %d wrong of 144\n", bad_v, bad_m, bad_4, bad_c);
  printf("12x12x12 product, one wave, s_memtime cycles (best of 20; the brackets alone: %llu, included below)\n", best[6]);
  printf("  valu      4 products (one per 16-lane row), 144 v_fmac_f64_dpp : %llu (%.1f per product)\n", best[0],
         best[0] / 4.0);
  printf("  mfma      1 product, 4 dependent 16x16x4 MFMAs (operands in MFMA maps): %llu\n", best[1]);
  printf("  mfma4     4 products, 16 MFMAs on 4 accumulators: %llu (%.1f per product)\n", best[2], best[2] / 4.0);
  printf("  mfma+cv   1 product with row<->MFMA layout conversions through LDS: %llu\n", best[3]);
  printf("  mfma_dep  16 dependent MFMAs: %llu (%.1f per MFMA)\n", best[4], best[4] / 16.0);
  printf("  valu_dep  144 dependent v_fmac_f64_dpp: %llu (%.2f per instruction)\n", best[5], best[5] / 144.0);
  return bad_v || bad_m || bad_c || bad_4;
}
