// Which source lane a DPP row_shl:6 / row_shr:6 / row_ror:10 move reads, on gfx950 (64-bit
// moves through __builtin_amdgcn_mov_dpp, as mpcq_engine.hip's dppd does).  Prints, for
// lanes 0..15 of row 0, the lane id each received.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int CTRL>
__device__ long long mv(long long v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
__global__ void k(long long* out) {
  const int l = threadIdx.x;
  const long long v = 1000 + l;
  out[l] = mv<0x106>(v);        // row_shl:6
  out[64 + l] = mv<0x116>(v);   // row_shr:6
  out[128 + l] = mv<0x12A>(v);  // row_ror:10
}
int main() {
  long long* d; hipMalloc(&d, 192 * 8);
  hipMemset(d, 0, 192 * 8);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  long long h[192]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[3] = {"row_shl:6", "row_shr:6", "row_ror:10"};
  for (int c = 0; c < 3; ++c) {
    printf("%-10s", nm[c]);
    for (int l = 0; l < 16; ++l) printf(" %lld", h[64 * c + l] - 1000);
    printf("\n");
  }
  return 0;
}
