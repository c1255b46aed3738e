// mpcq_planner.hip — batched FootstepPlanner for MI355X (gfx950): the producer
// of the engine's inputs (xref, fsteps), FootstepPlanner.py:76-425.
//
// One wave64 per instance (two per wave, one per 32-lane half, up to N = 31).  The
// per-instance state (gait table, xref, the rotation-command state machine) is read
// once, updated on chip and written once; every HBM row is moved by consecutive lanes.
//   roll               FootstepPlanner.py:401-425   lane-parallel row shift in LDS
//   compute_footsteps  FootstepPlanner.py:284-361   lane c < 12 walks column c of
//                                                   fsteps over the phases
//   getRefStates       FootstepPlanner.py:76-159    lane j owns xref column j (and
//                                                   column j + 64 for N = 64)
//
// Rounding follows numpy's evaluation order exactly (the oracle
// oracle/planner_oracle.c does the same and matches the reference bit for
// bit): no contraction of a*b+c into FMAs, except inside np.dot(R,
// next_footstep) whose BLAS kernel does use FMAs; cumsum left to right.
// Only cos/sin can differ (ocml vs the host libm) by an ulp.
#include <math.h>
#include <stdlib.h>

#include "mpcq_internal.h"

#pragma clang fp contract(off)

namespace mpcq {
namespace {

template <bool WIDE, int L>
struct PlanShared {
  alignas(16) double gait[100];
  alignas(16) double fs[260];
  // xref columns 1..N (lane j: columns j and j + 64); sized by the layout so the common
  // horizons keep the small LDS footprint
  double v6[WIDE ? 128 : L], v7[WIDE ? 128 : L];
  // per phase i of compute_footsteps: cos / sin of the yaw at the phase start and
  // the displacement dx, dy (FootstepPlanner.py:329-343), one lane per phase
  double ph_c[20], ph_s[20], ph_dx[20], ph_dy[20];
  // the instance's small inputs: state 0..11, v_ref 12..17, v_cur 18..23,
  // l_feet 24..35, h 36, h_rot 37
  double in[38];
  int flag, reduced, bad;
};

// LDS -> HBM in 16-B pieces per lane (n even, both sides 16-B aligned); L lanes per instance
template <int L>
__device__ __forceinline__ void copy_out16(double* dst, const double* src, int n, int ln) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    for (int e = ln; e < n / 2; e += L) reinterpret_cast<d2*>(dst)[e] = reinterpret_cast<const d2*>(src)[e];
  } else {  // a caller's buffer that is only 8-B aligned
    for (int e = ln; e < n; e += L) dst[e] = src[e];
  }
}

// numpy.linspace(a, b, n)[i] with endpoint: i * ((b - a) / (n - 1)) + a, last = b
__device__ __forceinline__ double linspace_at(double a, double b, int n, int i) {
  if (i == n - 1) return b;
  const double step = (b - a) / (double)(n - 1);
  return (double)i * step + a;
}

// The workgroup is one wave64, so an LDS hand-off between its lanes needs no hardware
// barrier (LDS is processed in order per wave): a compiler fence that keeps the LDS
// accesses on their side (also valid inside the half-wave branches of L = 32).
__device__ __forceinline__ void lane_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// WIDE: N + 1 > 64 xref columns (N = 64), lane j also owns column j + 64; a template
// parameter so the common horizons carry none of it (measured: 450 -> 340 M robots/s
// at N = 16 with the second column decided at run time, r03f).
// L: lanes per instance.  64: one instance per wave64; 32 (N + 1 <= 32): two instances
// per wave, one per half -- the phases are serial walks over the gait's 20 rows or the
// horizon's columns on a few lanes each (compute_footsteps 12, getRefStates N + 1), so
// the instruction stream, not HBM, bounded the kernel, and a half-wave instance halves
// it per instance (round 4).
template <bool WIDE, int L>
__global__ __launch_bounds__(64) void planner_kernel(mpcq_planner_params pp, PlanArgs a) {
  static_assert(L == 64 || (L == 32 && !WIDE), "64 lanes, or 32 without the second column");
  constexpr int RPW = 64 / L;
  __shared__ PlanShared<WIDE, L> shv[RPW];
  const int sub = L == 64 ? 0 : (int)(threadIdx.x >> 5);
  const int ln = L == 64 ? (int)threadIdx.x : (int)(threadIdx.x & 31);
  PlanShared<WIDE, L>& sh = shv[sub];
  const int64_t b = (int64_t)blockIdx.x * RPW + sub;
  if (b >= a.batch) return;  // (the other half, if any, runs on alone: no barrier below)
  const int N = a.N, NP = a.N + 1;
  double* gg = a.gait + b * 100;
  double* gx = a.xref + b * 12 * NP;
  const bool do_ref = a.ops & MPCQ_PLAN_REFSTATES, do_fs = a.ops & MPCQ_PLAN_FOOTSTEPS;

  // Every global read of the instance is issued here, before the first
  // LDS hand-off, so the wave pays one memory latency instead of one per phase.
  constexpr int GR = (100 + L - 1) / L;  // gait entries per lane
  double gv[GR];
#pragma unroll
  for (int q = 0; q < GR; ++q) gv[q] = ln + q * L < 100 ? gg[ln + q * L] : 0.0;
  double x[12];  // xref column `ln` (getRefStates rewrites only some rows)
  const bool col = do_ref && ln < NP;
#pragma unroll
  for (int r = 0; r < 12; ++r) x[r] = col ? gx[r * NP + ln] : 0.0;
  auto input = [&](int e) __attribute__((always_inline)) -> double {
    if (e < 12) return a.state[b * 12 + e];
    if (e < 18) return a.v_ref[b * 6 + e - 12];
    if (e < 24) return a.v_cur ? a.v_cur[b * 6 + e - 18] : a.state[b * 12 + e - 12];
    if (e < 36) return do_fs ? a.l_feet[b * 12 + e - 24] : 0.0;
    if (e == 36) return a.h ? a.h[b] : a.state[b * 12 + 2];
    return do_ref ? a.h_rot[b] : 0.0;  // e == 37
  };
  constexpr int IR = (38 + L - 1) / L;  // inputs per lane
  double iv[IR];
#pragma unroll
  for (int q = 0; q < IR; ++q) iv[q] = ln + q * L < 38 ? input(ln + q * L) : 0.0;
  if (ln == 0) sh.flag = do_ref ? a.rot_flag[b] : 0;
  if (ln == 1) sh.reduced = a.reduced ? a.reduced[b] : 0;
  if (ln == 2) sh.bad = 0;
#pragma unroll
  for (int q = 0; q < GR; ++q)
    if (ln + q * L < 100) sh.gait[ln + q * L] = gv[q];
#pragma unroll
  for (int q = 0; q < IR; ++q)
    if (ln + q * L < 38) sh.in[ln + q * L] = iv[q];
  lane_sync();
  const double* st = sh.in;
  const double* vr = sh.in + 12;
  // this instance's lanes of the wave (a ballot's bits)
  const uint64_t own = L == 64 ? ~0ull : (0xffffffffull << (32 * sub));

  // ---- roll (FootstepPlanner.py:401-425)
  if (a.ops & MPCQ_PLAN_ROLL) {
    const bool z = ln < 20 && sh.gait[5 * ln] == 0.0;
    const uint64_t zm = (__ballot(z) & own) >> (L == 64 ? 0 : 32 * sub);
    if (zm == 0) {
      if (ln == 0) sh.bad = 1;  // next(..., 0.0)[0] raises
    } else {
      const int index = __ffsll((unsigned long long)zm) - 1;
      const int last = (index + 19) % 20;  // gait[index - 1]; Python wraps -1
      bool same = true;
#pragma unroll
      for (int q = 1; q < 5; ++q) same = same && (sh.gait[q] == sh.gait[5 * last + q]);
      lane_sync();
      if (ln == 0) {
        if (same) {
          sh.gait[5 * last] += 1.0;
        } else {
          for (int q = 1; q < 5; ++q) sh.gait[5 * index + q] = sh.gait[q];
          sh.gait[5 * index] = 1.0;
        }
      }
      lane_sync();
      if (!(sh.gait[0] > 1.0)) {  // the current phase ends: shift the rows up
        // np.roll(gait, -1, axis=0) then a zero last row: element e <- e + 5
        double tv[GR];
#pragma unroll
        for (int q = 0; q < GR; ++q) {
          const int e = ln + q * L;
          tv[q] = e + 5 < 100 ? sh.gait[e + 5] : 0.0;
        }
        lane_sync();
#pragma unroll
        for (int q = 0; q < GR; ++q)
          if (ln + q * L < 100) sh.gait[ln + q * L] = tv[q];  // row 19 = 0
      } else {
        lane_sync();
        if (ln == 0) sh.gait[0] -= 1.0;
      }
      lane_sync();
    }
  }
  lane_sync();
  // ---- validity of compute_footsteps' walk: a terminator among rows 1..19
  if (a.ops & MPCQ_PLAN_FOOTSTEPS) {
    const bool z = ln >= 1 && ln < 20 && !(sh.gait[5 * ln] != 0.0);
    if ((__ballot(z) & own) == 0 && ln == 0) sh.bad = 1;  // self.gait[20, 0]: IndexError
  }
  lane_sync();
  if (sh.bad) {
    if (ln == 0 && a.status) a.status[b] = MPCQ_STATUS_BAD_GAIT;
    return;  // the instance's buffers stay as they were (the reference raised)
  }
  if (a.ops & MPCQ_PLAN_ROLL)
    copy_out16<L>(gg, sh.gait, 100, ln);

  // ---- compute_footsteps (FootstepPlanner.py:284-361)
  if (a.ops & MPCQ_PLAN_FOOTSTEPS) {
    const double* vc = sh.in + 18;
    const double h = sh.in[36];
    const int reduced = sh.reduced;
    for (int e = ln; e < 260; e += L) sh.fs[e] = (e % 13 == 0) ? sh.gait[5 * (e / 13)] : NAN;
    // the trigonometry of every phase in parallel (lane i = phase i), so the column
    // walk below carries no cos / sin on its sequential path; dt_cum is summed in
    // the reference's order (FootstepPlanner.py:310)
    if (ln >= 1 && ln < 20) {
      double dt_cum = 0.0;
      for (int i = 1; i <= ln; ++i) dt_cum += sh.gait[5 * (i - 1)] * pp.dt;
      const double angle = vr[5] * dt_cum;
      const double co = cos(angle), si = sin(angle);
      double dx, dy;
      if (vr[5] != 0.0) {
        dx = (vc[0] * si + vc[1] * (co - 1.0)) / vr[5];
        dy = (vc[1] * si - vc[0] * (co - 1.0)) / vr[5];
      } else {
        dx = vc[0] * dt_cum;
        dy = vc[1] * dt_cum;
      }
      sh.ph_c[ln] = co;
      sh.ph_s[ln] = si;
      sh.ph_dx[ln] = dx;
      sh.ph_dy[ln] = dy;
    }
    lane_sync();
    if (ln < 12) {
      const int c = ln, q = c / 3, r = c % 3;
      // next_footstep rows 0..1 of foot q: compute_next_footstep(v_ref, v_ref, h)
      // (FootstepPlanner.py:316, 363-399); row 2 is 0
      double nf[2];
      {
        const double cr0 = vr[1] * vr[5] - vr[2] * vr[4];  // np.cross(v_ref[0:3], v_ref[3:6])
        const double cr1 = vr[2] * vr[3] - vr[0] * vr[5];
        const double coef = 0.5 * sqrt(h / pp.g);
        const double half = pp.t_stance * 0.5;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          double v = 0.0 + half * vr[rr];
          v = v + pp.k_feedback * (vr[rr] - vr[rr]);
          v = v + coef * (rr == 0 ? cr0 : cr1);
          if (v > pp.L) v = pp.L;
          if (v < -pp.L) v = -pp.L;
          v = v + pp.shoulders[4 * rr + q];
          if (reduced) v = v - pp.reduced_offset[4 * rr + q];
          nf[rr] = v;
        }
      }
      // row 0: stance feet where they are (l_feet.ravel('F')[c] = l_feet[r][q])
      const double l0 = sh.gait[1 + q] == 1.0 ? sh.in[24 + 4 * r + q] : NAN;
      double prev = l0;  // fsteps[i-1, 1+c]
      sh.fs[1 + c] = l0;
      bool prev_st = sh.gait[1 + q] == 1.0;
      for (int i = 1; i < 20; ++i) {
        const double d = sh.gait[5 * i];
        if (!(d != 0.0)) break;
        const bool cur_st = sh.gait[5 * i + 1 + q] == 1.0;
        double v = NAN;
        if (prev_st && cur_st) {
          v = prev;
        } else if (!prev_st && cur_st) {
          const double co = sh.ph_c[i], si = sh.ph_s[i], dx = sh.ph_dx[i], dy = sh.ph_dy[i];
          // (R @ next_footstep)[r, q] + d[r]; R = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
          const double R0 = r == 0 ? co : (r == 1 ? si : 0.0);
          const double R1 = r == 0 ? -si : (r == 1 ? co : 0.0);
          const double R2 = r == 2 ? 1.0 : 0.0;
          double w = R0 * nf[0];
          w = fma(R1, nf[1], w);
          w = fma(R2, 0.0, w);
          v = w + (r == 0 ? dx : (r == 1 ? dy : 0.0));
        }
        sh.fs[13 * i + 1 + c] = v;
        prev = v;
        prev_st = cur_st;
      }
    }
    lane_sync();
    double* gf = a.fsteps + b * 260;
    copy_out16<L>(gf, sh.fs, 260, ln);
  }

  // ---- getRefStates (FootstepPlanner.py:76-159)
  // (N + 1 <= L: one column per lane; WIDE: the same arithmetic per column, lane j also
  // owning column j + 64)
  if constexpr (!WIDE) {
  if (a.ops & MPCQ_PLAN_REFSTATES) {
    const int j = ln;
    const double Tg = pp.T_gait, dt = pp.dt;
    if (col && j >= 1) {
      const double yaw = linspace_at(0.0, Tg - dt, N, j - 1) * vr[5];
      const double c = cos(yaw), s = sin(yaw);
      x[6] = vr[0] * c - vr[1] * s;
      x[7] = vr[0] * s + vr[1] * c;
      sh.v6[j] = x[6];
      sh.v7[j] = x[7];
    }
    lane_sync();
    if (col && j >= 1) {
      double a0 = 0.0, a1 = 0.0;  // np.cumsum: left to right
      for (int i = 1; i <= j; ++i) {
        a0 += sh.v6[i];
        a1 += sh.v7[i];
      }
      x[0] = dt * a0 + st[0];
      x[1] = dt * a1 + st[1];
      if (a.k == 0) x[2] = pp.h_ref;
      x[5] = vr[5] * linspace_at(dt, Tg, N, j - 1);
      x[11] = vr[5];
    }
    if (j == 0) {
#pragma unroll
      for (int r = 0; r < 12; ++r) x[r] = st[r];
    }
    // height / rotation command state machine (uniform per instance)
    int flag = sh.flag;
    double h_rot = sh.in[37];
    const double step = pp.cmd_threshold;
    const double v2 = vr[2];
    if (fabs(v2) > step && flag != 1) flag = 1;
    int branch = 0;
    if (fabs(v2) > step && flag == 1) {
      h_rot += v2 * dt;
      branch = 1;
    } else if (fabs(v2) < step && flag == 1) {
      flag = 2;
      branch = 2;
    } else if (flag == 0) {
      branch = 3;
    }
    if (col && j >= 1) {
      if (branch == 1) { x[2] = h_rot; x[8] = v2; }
      else if (branch == 2) { x[8] = 0.0; x[9] = 0.0; x[10] = 0.0; }
      else if (branch == 3) { x[2] = pp.h_ref; x[8] = 0.0; }
      if (flag != 0) {
        const double to = linspace_at(0.0, Tg - dt, N, j - 1);
        x[3] = st[3] + vr[3] * to;  // xref[3, 0] was just set to abg[0]
        x[4] = st[4] + vr[4] * to;
        x[9] = vr[3];
        x[10] = vr[4];
      }
    }
    if (col) {
#pragma unroll
      for (int r = 0; r < 12; ++r) gx[r * NP + j] = x[r];
    }
    if (ln == 0) {
      a.rot_flag[b] = flag;
      a.h_rot[b] = h_rot;
    }
  }
  } else {
  if (a.ops & MPCQ_PLAN_REFSTATES) {
    const double Tg = pp.T_gait, dt = pp.dt;
    // a second column per lane only when N + 1 > 64 (N = 64: column 64 on lane 0)
    const int j2 = ln + 64;
    const bool col2 = WIDE && do_ref && j2 < NP;
    double x2[12];
#pragma unroll
    for (int r = 0; r < 12; ++r) x2[r] = 0.0;
    if constexpr (WIDE) {
#pragma unroll
      for (int r = 0; r < 12; ++r) x2[r] = col2 ? gx[r * NP + j2] : 0.0;
    }
    auto velocities = [&](int j, bool on, double (&xx)[12]) __attribute__((always_inline)) {
      if (on && j >= 1) {
        const double yaw = linspace_at(0.0, Tg - dt, N, j - 1) * vr[5];
        const double c = cos(yaw), s = sin(yaw);
        xx[6] = vr[0] * c - vr[1] * s;
        xx[7] = vr[0] * s + vr[1] * c;
        sh.v6[j] = xx[6];
        sh.v7[j] = xx[7];
      }
    };
    velocities(ln, col, x);
    if constexpr (WIDE) velocities(j2, col2, x2);
    lane_sync();
    // height / rotation command state machine (uniform per instance)
    int flag = sh.flag;
    double h_rot = sh.in[37];
    const double step = pp.cmd_threshold;
    const double v2 = vr[2];
    if (fabs(v2) > step && flag != 1) flag = 1;
    int branch = 0;
    if (fabs(v2) > step && flag == 1) {
      h_rot += v2 * dt;
      branch = 1;
    } else if (fabs(v2) < step && flag == 1) {
      flag = 2;
      branch = 2;
    } else if (flag == 0) {
      branch = 3;
    }
    auto column = [&](int j, bool on, double (&xx)[12]) __attribute__((always_inline)) {
      if (on && j >= 1) {
        double a0 = 0.0, a1 = 0.0;  // np.cumsum: left to right
        for (int i = 1; i <= j; ++i) {
          a0 += sh.v6[i];
          a1 += sh.v7[i];
        }
        xx[0] = dt * a0 + st[0];
        xx[1] = dt * a1 + st[1];
        if (a.k == 0) xx[2] = pp.h_ref;
        xx[5] = vr[5] * linspace_at(dt, Tg, N, j - 1);
        xx[11] = vr[5];
      }
      if (j == 0) {
#pragma unroll
        for (int r = 0; r < 12; ++r) xx[r] = st[r];
      }
      if (on && j >= 1) {
        if (branch == 1) { xx[2] = h_rot; xx[8] = v2; }
        else if (branch == 2) { xx[8] = 0.0; xx[9] = 0.0; xx[10] = 0.0; }
        else if (branch == 3) { xx[2] = pp.h_ref; xx[8] = 0.0; }
        if (flag != 0) {
          const double to = linspace_at(0.0, Tg - dt, N, j - 1);
          xx[3] = st[3] + vr[3] * to;  // xref[3, 0] was just set to abg[0]
          xx[4] = st[4] + vr[4] * to;
          xx[9] = vr[3];
          xx[10] = vr[4];
        }
      }
      if (on) {
#pragma unroll
        for (int r = 0; r < 12; ++r) gx[r * NP + j] = xx[r];
      }
    };
    column(ln, col, x);
    if constexpr (WIDE) column(j2, col2, x2);
    if (ln == 0) {
      a.rot_flag[b] = flag;
      a.h_rot[b] = h_rot;
    }
  }
  }
  if (ln == 0 && a.status) a.status[b] = 0;
}

}  // namespace

// MPCQ_PLAN_LANES=64: one instance per wave64 at every horizon (A/B timing only; the
// results are identical)
int mpcq_plan_lanes() {
  static const int v = [] {
    const char* e = getenv("MPCQ_PLAN_LANES");
    return e && e[0] == '6' ? 64 : 32;
  }();
  return v;
}

hipError_t launch_plan(const mpcq_planner_params& pp, const PlanArgs& a, hipStream_t s) {
  if (a.batch <= 0) return hipSuccess;
  if (a.N < 1 || a.N > 64) return hipErrorInvalidValue;
  if (a.N + 1 > 64) {
    hipLaunchKernelGGL((planner_kernel<true, 64>), dim3((unsigned)a.batch), dim3(64), 0, s, pp, a);
  } else if (a.N + 1 > 32 || mpcq_plan_lanes() == 64) {
    hipLaunchKernelGGL((planner_kernel<false, 64>), dim3((unsigned)a.batch), dim3(64), 0, s, pp, a);
  } else {  // two instances per wave64
    hipLaunchKernelGGL((planner_kernel<false, 32>), dim3((unsigned)((a.batch + 1) / 2)), dim3(64), 0, s, pp, a);
  }
  return hipGetLastError();
}

}  // namespace mpcq
