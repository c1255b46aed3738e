// mpcq_session.hip — the per-tick epilogue of a closed-loop session on MI355X:
// everything MPC.run and the Logger do with the QP solution after the solve,
// plus the state the next tick starts from.  One wave64 per robot.
//
//   x_robot = x[:12N] (12 x N, Fortran order) + xref[:, 1:]   MPC.py:432-449
//   q_w += R(q_w[5]) q_next[0:2], ...                          MPC.py:503-510
//   cost components (diag(x) diag(P) x, summed per state and   Logger.py:406-418
//   for the forces, numpy's pairwise summation)
//   next warm start: states shifted one stage (last zeroed),   MPC.py:403-406
//   forces rolled by one stage with wrap-around
//   virtual robot: the next tick's state / feet from x_robot[:, 0]
//   (processing.py:33-38, Interface.py:100-138)
//
// Rounding follows numpy: no contraction except np.dot(R, q_next[0:2]),
// which numpy evaluates as fma(R[i,0], q0, R[i,1] * q1).
#include <math.h>

#include "mpcq_internal.h"

#pragma clang fp contract(off)

namespace mpcq {
namespace {

// numpy's pairwise_sum (umath loops: 8 partial sums below 128 elements,
// halves rounded to a multiple of 8 above), on a strided LDS array
template <int n>
__device__ __forceinline__ double pairwise(const double* v, int stride) {
  if constexpr (n < 8) {
    double s = -0.0;
    for (int i = 0; i < n; ++i) s += v[i * stride];
    return s;
  } else if constexpr (n <= 128) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = v[j * stride];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += v[(i + j) * stride];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += v[i * stride];
    return res;
  } else {
    constexpr int n2 = n / 2 - (n / 2) % 8;
    return pairwise<n2>(v, stride) + pairwise<n - n2>(v + n2 * stride, stride);
  }
}

template <int N>
__global__ __launch_bounds__(64) void retrieve_kernel(SessionArgs a) {
  constexpr int n = 24 * N, NP = N + 1;
  __shared__ double xs[n];
  __shared__ double cost[n];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (b >= a.batch) return;
  const double* gx = a.x + b * n;
  const double* xr = a.xref + b * 12 * NP;
  const int st = a.status[b];
  // a robot whose planner failed this tick (where the reference raises) is treated
  // like a failed solve: it keeps its pose and virtual state and restarts cold
  const bool failed = !(st == MPCQ_STATUS_SOLVED || st == MPCQ_STATUS_SOLVED_INACCURATE ||
                        st == MPCQ_STATUS_MAX_ITER_REACHED) || a.plan_status[b] != 0;
  for (int e = lane; e < n; e += 64) {
    const double v = gx[e];
    xs[e] = v;
    const double w = e < 12 * N ? a.state_weights[e % 12] : a.force_weight;
    cost[e] = (v * w) * v;  // (diag(x) @ diag(P)) @ x
  }
  __syncthreads();
  // x_robot [12][N] and the next warm start
  double* xo = a.x_robot + b * 12 * N;
  for (int e = lane; e < 12 * N; e += 64) {
    const int r = e / N, k = e % N;
    xo[e] = xs[12 * k + r] + xr[r * NP + k + 1];
  }
  double* wx = a.warm_x + b * n;
  for (int e = lane; e < n; e += 64) {
    double v;
    if (e < 12 * N) v = e < 12 * (N - 1) ? xs[e + 12] : 0.0;
    else v = xs[12 * N + (e - 12 * N + 12) % (12 * N)];
    wx[e] = failed ? 0.0 : v;  // a failed solve restarts cold (osqp would carry NaNs)
  }
  if (failed) {
    double* yy = a.y + b * 44 * N;
    for (int e = lane; e < 44 * N; e += 64) yy[e] = 0.0;
    if (lane == 0) a.rho[b] = a.rho0;
  }
  // cost components: lanes 0..11 the states, lane 12 the forces
  if (lane < 12) a.cost[b * 13 + lane] = pairwise<N>(cost + lane, 12);
  if (lane == 12) a.cost[b * 13 + 12] = pairwise<12 * N>(cost + 12 * N, 1);
  if (lane == 0 && a.plan_status[b] != 0) a.status[b] = a.plan_status[b];
  if (lane == 0 && !failed) {  // a failed robot keeps its pose and virtual state
    // q_next = x_robot[0:6, 0], v_next = x_robot[6:12, 0]
    double qn[12];
#pragma unroll
    for (int r = 0; r < 12; ++r) qn[r] = xs[r] + xr[r * NP + 1];
    double* qw = a.q_w + b * 6;
    const double c = cos(qw[5]), s = sin(qw[5]);
    const double d0 = fma(c, qn[0], (-s) * qn[1]);
    const double d1 = fma(s, qn[0], c * qn[1]);
    qw[0] = qw[0] + d0;
    qw[1] = qw[1] + d1;
    qw[2] = qn[2];
    qw[3] = qn[3];
    qw[4] = qn[4];
    qw[5] = qw[5] + qn[5];
    // virtual robot: new local frame under the predicted base, yaw removed
    const double cy = cos(qn[5]), sy = sin(qn[5]);
    double* ns = a.next_state + b * 12;
    ns[0] = 0.0;
    ns[1] = 0.0;
    ns[2] = qn[2];
    ns[3] = qn[3];
    ns[4] = qn[4];
    ns[5] = 0.0;
    ns[6] = cy * qn[6] + sy * qn[7];
    ns[7] = -sy * qn[6] + cy * qn[7];
    ns[8] = qn[8];
    ns[9] = cy * qn[9] + sy * qn[10];
    ns[10] = -sy * qn[9] + cy * qn[10];
    ns[11] = qn[11];
    // feet: the phase that will be current after the next roll holds the
    // positions of the feet then in stance (row 0 if the phase goes on, row 1
    // if it ends); swing feet sit under their shoulders
    const double* fs = a.fsteps + b * 260;
    const double* gt = a.gait + b * 100;
    const int row = gt[0] > 1.0 ? 0 : 1;
    double* lf = a.next_l_feet + b * 12;
    for (int q = 0; q < 4; ++q) {
      double px = fs[13 * row + 1 + 3 * q], py = fs[13 * row + 2 + 3 * q], pz = fs[13 * row + 3 + 3 * q];
      if (isnan(px) || isnan(py) || isnan(pz)) {
        px = a.shoulders[q] + qn[0];
        py = a.shoulders[4 + q] + qn[1];
        pz = 0.0;
      }
      const double dx = px - qn[0], dy = py - qn[1];
      lf[q] = cy * dx + sy * dy;
      lf[4 + q] = -sy * dx + cy * dy;
      lf[8 + q] = pz;
    }
  }
}

// Longest-first dispatch order from the iteration counts of the tick just solved
// (one workgroup; counting sort over buckets of 16 iterations, LDS atomics, so the
// order inside a bucket is arbitrary -- every instance's result is independent of
// the workgroup that solves it).  A robot's warm-started count predicts its next
// one (tools/tick_iters.py), and index-order dispatch puts long solves that land
// late in the launch on its critical path.
constexpr int kOrderBuckets = 256;
__global__ __launch_bounds__(1024) void order_kernel(const int32_t* __restrict__ iters, int64_t B,
                                                     int32_t* __restrict__ order) {
  __shared__ int hist[kOrderBuckets];
  const int t = threadIdx.x;
  auto bucket = [](int32_t it) { const int q = (it > 0 ? it : 0) >> 4; return q < kOrderBuckets - 1 ? q : kOrderBuckets - 1; };
  if (t < kOrderBuckets) hist[t] = 0;
  __syncthreads();
  for (int64_t i = t; i < B; i += blockDim.x) atomicAdd(&hist[bucket(iters[i])], 1);
  __syncthreads();
  if (t == 0) {  // exclusive offsets, the longest bucket first
    int acc = 0;
    for (int q = kOrderBuckets - 1; q >= 0; --q) {
      const int h = hist[q];
      hist[q] = acc;
      acc += h;
    }
  }
  __syncthreads();
  for (int64_t i = t; i < B; i += blockDim.x) order[atomicAdd(&hist[bucket(iters[i])], 1)] = (int32_t)i;
}

}  // namespace

hipError_t launch_order(const int32_t* iters, int64_t batch, int32_t* order, hipStream_t s) {
  if (batch <= 0) return hipSuccess;
  if (batch > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, s, iters, batch, order);
  return hipGetLastError();
}

hipError_t launch_retrieve(int N, const SessionArgs& a, hipStream_t s) {
  if (a.batch <= 0) return hipSuccess;
  switch (N) {
#define MPCQ_RET_CASE(NN) \
    case NN: hipLaunchKernelGGL(retrieve_kernel<NN>, dim3((unsigned)a.batch), dim3(64), 0, s, a); break;
    MPCQ_HORIZONS(MPCQ_RET_CASE)
#undef MPCQ_RET_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mpcq
