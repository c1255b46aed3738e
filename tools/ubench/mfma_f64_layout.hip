// Checks the v_mfma_f64_16x16x4_f64 operand / result lane maps the Kinv formation
// (mpcq_engine.hip, kinv_form) relies on, with exact integer data and an asymmetric B:
//   A[i][k] from lane l = i + 16 k (i = l & 15, k = l >> 4), B[k][j] from lane l = j + 16 k,
//   D[i][j]: lane l = j + 16 (i & 3), register i >> 2  (row (l >> 4) + 4 r, column l & 15),
// and that register s of a result, used as the next product's B operand, is K-slice s.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/mfl tools/ubench/mfma_f64_layout.hip && /tmp/mfl
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(const double* A, const double* B, const double* C, double* D, double* D2) {
  const int l = threadIdx.x;
  // one 16x16x4 product: A 16x4, B 4x16, C 16x16
  d4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[16 * ((l >> 4) + 4 * r) + (l & 15)];
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[4 * (l & 15) + (l >> 4)], B[16 * (l >> 4) + (l & 15)], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[16 * ((l >> 4) + 4 * r) + (l & 15)] = d[r];
  // chained: D2 = A16 (16x16, as 4 K-slices) * d (16x16, the previous result as B) + 0
  d4 z = {0.0, 0.0, 0.0, 0.0};
  for (int s = 0; s < 4; ++s) z = __builtin_amdgcn_mfma_f64_16x16x4f64(C[16 * (l & 15) + 4 * s + (l >> 4)], d[s], z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D2[16 * ((l >> 4) + 4 * r) + (l & 15)] = z[r];
}

int main() {
  double hA[64], hB[64], hC[256], hD[256], hD2[256], ref[256], ref2[256];
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) hA[4 * i + k] = (i * 7 + k * 3) % 11 - 5;
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) hB[16 * k + j] = (k * 5 + j * j) % 13 - 6;
  for (int i = 0; i < 256; ++i) hC[i] = (i * 29) % 17 - 8;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = hC[16 * i + j];
      for (int k = 0; k < 4; ++k) s += hA[4 * i + k] * hB[16 * k + j];
      ref[16 * i + j] = s;
    }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += hC[16 * i + k] * ref[16 * k + j];
      ref2[16 * i + j] = s;
    }
  double *dA, *dB, *dC, *dD, *dD2;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC); hipMalloc(&dD, sizeof hD);
  hipMalloc(&dD2, sizeof hD2);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, dD2);
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  hipMemcpy(hD2, dD2, sizeof hD2, hipMemcpyDeviceToHost);
  int bad = 0, bad2 = 0;
  for (int i = 0; i < 256; ++i) { bad += hD[i] != ref[i]; bad2 += hD2[i] != ref2[i]; }
  printf("mfma_f64_16x16x4 layout: %d / 256 wrong; chained (result as B): %d / 256 wrong\n", bad, bad2);
  return bad || bad2;
}
