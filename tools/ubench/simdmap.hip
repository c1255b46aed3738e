// Where the waves of co-resident workgroups land on gfx950: B workgroups of 256
// threads with ~77 KB of dynamic LDS each (two per CU, as the N = 16 engine) spin for
// a fixed time; each wave records its HW_ID (SIMD, CU, SE, ...) and XCC_ID.  The host
// groups the workgroups by CU and prints, per CU, which blocks shared it and the SIMD
// of each of their waves (is the engine's sweep wave 0 of two co-resident instances
// on the same SIMD?).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <map>
#include <vector>
#include <tuple>
__global__ void k(unsigned* out, long long spin) {
  extern __shared__ double lds[];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    out[(blockIdx.x * 4 + w) * 2] = hw;
    out[(blockIdx.x * 4 + w) * 2 + 1] = xcc;
  }
  lds[threadIdx.x] = 1.0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 100000; ++i)  // bounded: ~spin cycles
    if (__builtin_amdgcn_s_memtime() - t0 > spin) break;
  __syncthreads();
}
int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 512;
  unsigned* d;
  hipMalloc(&d, (size_t)B * 4 * 2 * 4);
  hipMemset(d, 0, (size_t)B * 4 * 2 * 4);
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 77 * 1024) != hipSuccess)
    printf("attribute refused\n");
  hipLaunchKernelGGL(k, dim3(B), dim3(256), 77 * 1024, 0, d, 2000000LL);
  const hipError_t e = hipDeviceSynchronize();
  printf("launch: %s\n", hipGetErrorString(hipGetLastError() != hipSuccess ? hipErrorUnknown : e));
  std::vector<unsigned> h((size_t)B * 8);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  std::map<std::tuple<unsigned, unsigned, unsigned, unsigned>, std::vector<int>> cu;
  for (int b = 0; b < B; ++b) {
    const unsigned hw = h[b * 8], xcc = h[b * 8 + 1] & 0xF;
    const unsigned cu_id = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    cu[{xcc, se, sh, cu_id}].push_back(b);
  }
  int same = 0, pairs = 0, shown = 0;
  for (auto& kv : cu) {
    auto& v = kv.second;
    if (shown < 12) {
      printf("xcc %u se %u sh %u cu %2u:", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first),
             std::get<3>(kv.first));
      for (int b : v) {
        printf("  blk %4d simd", b);
        for (int w = 0; w < 4; ++w) printf(" %u", (h[(b * 4 + w) * 2] >> 4) & 3);
        printf(" tg %u", (h[b * 8] >> 16) & 0xF);
      }
      printf("\n");
      ++shown;
    }
    for (size_t i = 0; i < v.size(); ++i)
      for (size_t j = i + 1; j < v.size(); ++j) {
        ++pairs;
        same += ((h[v[i] * 8] >> 4) & 3) == ((h[v[j] * 8] >> 4) & 3);
      }
  }
  printf("%zu CUs, %d co-resident pairs, %d with wave 0 on the same SIMD\n", cu.size(), pairs, same);
  return 0;
}
