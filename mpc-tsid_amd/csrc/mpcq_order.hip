// mpcq_order.hip — dispatch order of a batch solve by gait class (MPCQ_FLAG_ORDER_BY_CLASS).
//
// The hardware hands out an engine launch's workgroups in index order, so a long solve
// that lands in a late dispatch round ends the launch late.  A cold batch
// has no previous tick to rank it by (the session path orders by the last tick's counts,
// mpcq_session.hip order_kernel), and no sampled input predicts a trot QP's iteration count
// (tools/iter_predictors.py) -- but the gait does, across gaits: on a C5 shard (trot / bound
// / pace) trot solves take 886 iterations on average and up to 3100, bound and pace ~600
// and up to ~1000 (Spearman -0.63, profiles/r06_iter_predictors.txt).  So:
//   class_kernel      : per instance, its gait class: the set of contact masks its fsteps
//                       phases use (MPC.py:635-652's contact rule), a 16-bit bitmap, folded
//                       into one of kSlots slots of the context's class table;
//   class_order_kernel: one workgroup: each instance's expected cost = the mean iteration
//                       count its class slot has seen in earlier launches on this context
//                       (the mean over every seen slot for a new class, 0 before any
//                       launch), in buckets of 16 iterations; a stable counting sort, the
//                       most expensive bucket first, index order inside a bucket (a batch of
//                       one class keeps the identity order);
//   class_learn_kernel: after the engine, each instance's iteration count into its slot.
// Every instance's result is independent of the workgroup that solves it, so the order
// changes no result bit (tests/test_gpu_order.py).
// suspended_kernel (sliced solves, mpcq_set_slice): the instances a launch suspended, the
// farthest from convergence first, for the next launch.
#include <stdint.h>

#include "mpcq_internal.h"

namespace mpcq {
namespace {

constexpr int kSlots = 251;     // class table slots (a prime: the bitmap modulo it)
constexpr int kBuckets = 256;   // expected-cost buckets of 16 iterations
constexpr int kWaves = 16;      // the order kernel's workgroup: 1024 threads

__device__ __forceinline__ int class_slot(const double* __restrict__ fs) {
  unsigned key = 0;
  for (int j = 0; j < 20; ++j) {
    const double d = fs[13 * j];
    if (d == 0.0) return (int)(key % kSlots);
    unsigned msk = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double x = fs[13 * j + 1 + 3 * q];
      msk |= (!(isnan(x) || x == 0.0) ? 1u : 0u) << q;
    }
    key |= 1u << msk;
  }
  return 0;  // no terminating row: the engine reports BAD_GAIT, any slot will do
}

__global__ __launch_bounds__(256) void class_kernel(const double* __restrict__ fsteps, int64_t B,
                                                    int32_t* __restrict__ cls) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) cls[i] = class_slot(fsteps + i * 260);
}

__global__ __launch_bounds__(1024) void class_order_kernel(const int32_t* __restrict__ cls, int64_t B,
                                                           const unsigned long long* __restrict__ sum,
                                                           const unsigned* __restrict__ cnt,
                                                           int32_t* __restrict__ order) {
  __shared__ int cost[kSlots];          // bucket of each slot
  __shared__ int base[kBuckets];        // next free position of each bucket
  __shared__ int wcnt[kWaves][kBuckets];
  __shared__ unsigned long long tot_s, tot_n;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  if (t == 0) { tot_s = 0; tot_n = 0; }
  if (t < kBuckets) base[t] = 0;
  __syncthreads();
  unsigned long long my_s = 0, my_n = 0;
  if (t < kSlots) {
    my_s = sum[t];
    my_n = cnt[t];
    if (my_n) { atomicAdd(&tot_s, my_s); atomicAdd(&tot_n, my_n); }
  }
  __syncthreads();
  if (t < kSlots) {  // (the mean over every seen slot for a class not seen yet)
    const unsigned long long e = my_n ? my_s / my_n : (tot_n ? tot_s / tot_n : 0);
    const unsigned long long q = e >> 4;
    cost[t] = q < kBuckets - 1 ? (int)q : kBuckets - 1;
  }
  __syncthreads();
  for (int64_t i = t; i < B; i += blockDim.x) atomicAdd(&base[cost[cls[i]]], 1);
  __syncthreads();
  if (w == 0) {  // exclusive offsets, the most expensive bucket first: four buckets per lane
    int h[4], run = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) { h[j] = base[kBuckets - 1 - (4 * lane + j)]; run += h[j]; }
    int inc = run;  // inclusive scan of the lanes' sums
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o);
      if (lane >= o) inc += v;
    }
    int acc = inc - run;
#pragma unroll
    for (int j = 0; j < 4; ++j) { base[kBuckets - 1 - (4 * lane + j)] = acc; acc += h[j]; }
  }
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int64_t c0 = 0; c0 < B; c0 += blockDim.x) {
    for (int e = t; e < kWaves * kBuckets; e += blockDim.x) (&wcnt[0][0])[e] = 0;
    __syncthreads();
    const int64_t i = c0 + t;
    const int q = i < B ? cost[cls[i]] : -1;
    // rank among the earlier lanes of this wave with the same bucket; per-bucket counts
    int rank = 0;
    bool done = q < 0;
    for (;;) {
      const unsigned long long pend = __ballot(!done);
      if (!pend) break;
      const int leader = __ffsll((long long)pend) - 1;
      const int ql = __shfl(q, leader);
      const unsigned long long m = __ballot(!done && q == ql);
      if (!done && q == ql) {
        rank = __popcll(m & below);
        done = true;
      }
      if (lane == leader) wcnt[w][ql] = __popcll(m);
    }
    __syncthreads();
    if (t < kBuckets) {  // waves in order: each wave's start inside the bucket
      int run = base[t];
#pragma unroll
      for (int v = 0; v < kWaves; ++v) {
        const int h = wcnt[v][t];
        wcnt[v][t] = run;
        run += h;
      }
      base[t] = run;
    }
    __syncthreads();
    if (q >= 0) order[wcnt[w][q] + rank] = (int32_t)i;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void class_learn_kernel(const int32_t* __restrict__ cls,
                                                          const int32_t* __restrict__ iters, int64_t B,
                                                          unsigned long long* __restrict__ sum,
                                                          unsigned* __restrict__ cnt) {
  // a batch holds few classes: sum in LDS per block, then one global atomic per class and block
  __shared__ unsigned long long bs[kSlots];
  __shared__ unsigned bn[kSlots];
  const int t = threadIdx.x;
  for (int q = t; q < kSlots; q += blockDim.x) { bs[q] = 0; bn[q] = 0; }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + t;
  if (i < B) {
    const int32_t it = iters[i];
    if (it > 0) {
      atomicAdd(&bs[cls[i]], (unsigned long long)it);
      atomicAdd(&bn[cls[i]], 1u);
    }
  }
  __syncthreads();
  for (int q = t; q < kSlots; q += blockDim.x)
    if (bn[q]) {
      atomicAdd(&sum[q], bs[q]);
      atomicAdd(&cnt[q], bn[q]);
    }
}

// Sliced solves (mpcq_set_slice): the suspended instances of the last launch for the next one,
// the largest key first -- the iterations left, extrapolated from the residuals' decay over the
// second half of the slice (Spearman +0.995 with the final iteration count over C3's instances
// suspended at 1200 iterations, tools/resume_predictors.py) -- in buckets of 1/8 octave, the last
// launch's order inside a bucket: a stable counting sort in one workgroup (the class order's
// scheme)
__device__ __forceinline__ int key_bucket(double v) {
  if (!(v > 0.0)) return 0;
  const double e = floor(8.0 * log2(v)) + 128.0;  // (1/8 octave; keys from 2^-16 to 2^16)
  return e < 0.0 ? 0 : (e > kBuckets - 1.0 ? kBuckets - 1 : (int)e);
}

__global__ __launch_bounds__(1024) void suspended_kernel(const int32_t* __restrict__ prev, int64_t n,
                                                         const int32_t* __restrict__ status,
                                                         const double* __restrict__ key,
                                                         int32_t* __restrict__ list, int32_t* __restrict__ count) {
  __shared__ int base[kBuckets];
  __shared__ int wcnt[kWaves][kBuckets];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  if (t < kBuckets) base[t] = 0;
  __syncthreads();
  for (int64_t i = t; i < n; i += blockDim.x) {
    const int32_t id = prev ? prev[i] : (int32_t)i;
    if (status[id] == kStatusSuspended) atomicAdd(&base[key_bucket(key[2 * id])], 1);
  }
  __syncthreads();
  if (w == 0) {  // exclusive offsets, the largest key first (four buckets per lane)
    int h[4], run = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) { h[j] = base[kBuckets - 1 - (4 * lane + j)]; run += h[j]; }
    int inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o);
      if (lane >= o) inc += v;
    }
    if (lane == 63) *count = inc;  // (the total)
    int acc = inc - run;
#pragma unroll
    for (int j = 0; j < 4; ++j) { base[kBuckets - 1 - (4 * lane + j)] = acc; acc += h[j]; }
  }
  __syncthreads();
  for (int64_t c0 = 0; c0 < n; c0 += blockDim.x) {
    for (int e = t; e < kWaves * kBuckets; e += blockDim.x) (&wcnt[0][0])[e] = 0;
    __syncthreads();
    const int64_t i = c0 + t;
    int32_t id = -1;
    int q = -1;
    if (i < n) {
      id = prev ? prev[i] : (int32_t)i;
      if (status[id] == kStatusSuspended) q = key_bucket(key[2 * id]);
    }
    int rank = 0;
    bool done = q < 0;
    for (;;) {
      const unsigned long long pend = __ballot(!done);
      if (!pend) break;
      const int leader = __ffsll((long long)pend) - 1;
      const int ql = __shfl(q, leader);
      const unsigned long long m = __ballot(!done && q == ql);
      if (!done && q == ql) {
        rank = __popcll(m & below);
        done = true;
      }
      if (lane == leader) wcnt[w][ql] = __popcll(m);
    }
    __syncthreads();
    if (t < kBuckets) {
      int run = base[t];
#pragma unroll
      for (int v = 0; v < kWaves; ++v) {
        const int h = wcnt[v][t];
        wcnt[v][t] = run;
        run += h;
      }
      base[t] = run;
    }
    __syncthreads();
    if (q >= 0) list[wcnt[w][q] + rank] = id;
    __syncthreads();
  }
}

}  // namespace

int class_table_slots() { return kSlots; }

hipError_t launch_suspended(const int32_t* prev, int64_t n, const int32_t* status, const double* key,
                            int32_t* list, int32_t* count, hipStream_t s) {
  if (n <= 0 || n > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(suspended_kernel, dim3(1), dim3(1024), 0, s, prev, n, status, key, list, count);
  return hipGetLastError();
}

hipError_t launch_class_order(const double* fsteps, int64_t B, int32_t* cls, const uint64_t* sum,
                              const uint32_t* cnt, int32_t* order, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (B > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(class_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, fsteps, B, cls);
  hipLaunchKernelGGL(class_order_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)cls, B,
                     (const unsigned long long*)sum, (const unsigned*)cnt, order);
  return hipGetLastError();
}

hipError_t launch_class_learn(const int32_t* cls, const int32_t* iters, int64_t B, uint64_t* sum, uint32_t* cnt,
                              hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(class_learn_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, cls, iters, B,
                     (unsigned long long*)sum, (unsigned*)cnt);
  return hipGetLastError();
}

}  // namespace mpcq
