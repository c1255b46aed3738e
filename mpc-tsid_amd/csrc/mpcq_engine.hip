// mpcq_engine.hip — batched convex-MPC QP engine for MI355X (gfx950, CDNA4).
//
// One workgroup of N/16 wave64s owns one QP instance for its whole life:
// formulation (MPC.py:98-378), Ruiz scaling, KKT factorisation and the
// OSQP-0.6 ADMM iterations run out of registers + LDS.  HBM sees only the
// compulsory inputs (xref, fsteps) and outputs (f0 / x / y / status).
//
// Layout: thread t = 4k + q owns stage k (forces f_k, states X^k := X_{k+1})
// quarter q: force columns 3q..3q+2 (= foot q), state columns 3q..3q+2, the
// dynamics rows 3q..3q+2, swing rows 3q..3q+2 and the five friction rows of
// foot q.  Its ADMM vectors (x, z, y, bounds, scaling) live in registers, as
// do rows 3q..3q+2 of the two 12x12 inverses below.
//
// KKT solve (P + sigma I + A' R A) w = b.  In stage order the matrix is block
// tridiagonal; the forces only couple inside a stage, so they are eliminated
// first (all stages in parallel, 12x12 per stage, F_k = K_ff,k^{-1} held by
// the stage's quad), which leaves a block-tridiagonal system in the states
// with 12x12 blocks:
//   D_k = K_XX,k - diag(Xd) Q_k diag(Xd) - diag(Hd_{k+1}) Q_{k+1} diag(Hd_{k+1})
//   L_k = C_X,k  - diag(Xd) Q_k diag(Hd_k)          Q_k = W_k' F_k W_k  (6x6)
// (W_k = B_k' diag(rho) on the velocity rows, the only rows where forces and
// states meet).  Block LDL': S_k = D_k - G_k L_k', G_k = L_k S_{k-1}^{-1}.
// Per ADMM iteration:
//   u = F b_f, beta = rho B u        (parallel)       bt_X = b_X - K_Xf u - ...
//   y_k = bt_k - G_k y_{k-1}          (sequential, 12x12, wave 0, 48 lanes)
//   w_k = S_k^{-1} y_k                (parallel)
//   X_k = w_k - G_{k+1}' X_{k+1}      (sequential)
//   f_k = F_k (b_f - W_k gamma_k)     (parallel)
// Everything else (A x, A' y, projections, residuals) is per stage.
#include <math.h>

#include "mpcq_internal.h"

namespace mpcq {
namespace {

constexpr double kInf = 1e30;  // OSQP_INFTY
constexpr double kMinScaling = 1e-4, kMaxScaling = 1e4;
constexpr double kRhoMin = 1e-6, kRhoMax = 1e6, kRhoEq = 1e3, kRhoTol = 1e-4;
constexpr double kDivTol = 1e-30;

// constraint classes -> rho (OSQP set_rho_vec; polish uses 3 / 4)
enum : int { RC_LOOSE = 0, RC_INEQ = 1, RC_EQ = 2, RC_POL_ACT = 3, RC_POL_OFF = 4 };

#ifdef MPCQ_STAMPS
#define STAMP_DECL uint64_t st_acc[16] = {}; uint64_t st_last = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { if (threadIdx.x == 0) { const uint64_t nw_ = __builtin_amdgcn_s_memtime(); st_acc[i] += nw_ - st_last; st_last = nw_; } } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// CSC offsets of MPC.create_ML's pattern (see mpcq_pattern in mpcq_api.cpp).
template <int N>
__device__ __forceinline__ int XO(int k, int i) {  // state column X^k[i] (= X_{k+1}[i])
  return (k < N - 1) ? 30 * k + (i < 6 ? 2 * i : 12 + 3 * (i - 6)) : 30 * (N - 1) + i;
}
template <int N>
__device__ __forceinline__ int FO(int k, int f, int c) {  // force column f_k[3f+c]
  return 30 * N - 18 + 96 * k + 24 * f + 7 * c;
}

// ---------------------------------------------------------------------------
// cross-lane helpers

__device__ __forceinline__ void wave_sync() {
  // LDS is processed in order per wave, so a wave-wide hand-off through LDS
  // needs no hardware barrier; the asm memory clobber stops the compiler from
  // moving (or hoisting out of loops) LDS accesses across this point.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int NW>
__device__ __forceinline__ void sync_all() {
  if constexpr (NW == 1) wave_sync();
  else __syncthreads();
}

template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)bits, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(bits >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// quad_perm controls
constexpr int QX1 = 0xB1, QX2 = 0x4E;
template <int J>
__device__ __forceinline__ double qbcast(double v) { return dppd<85 * J>(v); }
__device__ __forceinline__ double quad_sum(double v) {
  v += dppd<QX1>(v);
  v += dppd<QX2>(v);
  return v;
}
// the stage's 12-vector from the 3 entries each quad lane holds (all lanes active)
__device__ __forceinline__ void quad_gather12(const double (&own)[3], double (&all)[12]) {
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    all[0 + e] = qbcast<0>(own[e]);
    all[3 + e] = qbcast<1>(own[e]);
    all[6 + e] = qbcast<2>(own[e]);
    all[9 + e] = qbcast<3>(own[e]);
  }
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------------------
// Formulation pieces (restating MPC.py; oracle/mpcq_oracle.c is the CPU twin)

__device__ __forceinline__ void inv3(const double* M, double* R) {
  const double a = M[0], b = M[1], c = M[2], d = M[3], e = M[4], f = M[5], g = M[6], h = M[7],
               i = M[8];
  const double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
  const double det = a * A + b * B + c * C;
  const double id = 1.0 / det;
  R[0] = A * id; R[1] = -(b * i - c * h) * id; R[2] = (b * f - c * e) * id;
  R[3] = B * id; R[4] = (a * i - c * g) * id;  R[5] = -(a * f - c * d) * id;
  R[6] = C * id; R[7] = -(a * h - b * g) * id; R[8] = (a * e - b * d) * id;
}

// The 24 CSC values of one foot's three force columns in one stage: dt/m row,
// B rows 9..11 = dt inv(Rz(yaw) gI) [lever]x (MPC.py:339-345), swing flag S
// (MPC.py:628), friction-cone coefficients (MPC.py:136-148).
__device__ __forceinline__ void form_foot(const mpcq_params& p, double yaw, double l0, double l1, double l2,
                          double swing, double* out) {
  const double cy = cos(yaw), sy = sin(yaw);
  const double R[9] = {cy, -sy, 0.0, sy, cy, 0.0, 0.0, 0.0, 1.0};
  double M[9], Mi[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int t = 0; t < 3; ++t)
      M[3 * r + t] = R[3 * r + 0] * p.gI[0 * 3 + t] + R[3 * r + 1] * p.gI[1 * 3 + t] +
                     R[3 * r + 2] * p.gI[2 * 3 + t];
  inv3(M, Mi);
  const double S[9] = {0.0, -l2, l1, l2, 0.0, -l0, -l1, l0, 0.0};
  const double dtm = p.dt / p.mass;
  int pos = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    out[pos++] = dtm;
#pragma unroll
    for (int r = 0; r < 3; ++r)
      out[pos++] = p.dt * (Mi[3 * r + 0] * S[0 * 3 + c] + Mi[3 * r + 1] * S[1 * 3 + c] +
                           Mi[3 * r + 2] * S[2 * 3 + c]);
    out[pos++] = swing;
    if (c < 2) {
      out[pos++] = 1.0;
      out[pos++] = -1.0;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) out[pos++] = -p.mu;
      out[pos++] = -1.0;
    }
  }
}

// Bounds of dynamics row (k, r) (MPC.py:197-221, 366-378, 410); xr = xref staged in LDS.
template <int N>
__device__ __forceinline__ double dyn_bound(const mpcq_params& p, const double* xr, int k, int r) {
  constexpr int NP1 = N + 1;
  double v = (r == 8) ? -(-p.gravity * p.dt) : -0.0;
  if (k == 0) {
    double ax0 = -xr[r * NP1];
    if (r < 6) ax0 = ax0 + p.dt * (-xr[(r + 6) * NP1]);
    v = v + ax0;
  }
  double dv;
  if (k >= 1) {
    dv = -xr[r * NP1 + k];
    if (r < 6) dv = dv + (-p.dt) * xr[(r + 6) * NP1 + k];
    dv = dv + xr[r * NP1 + k + 1];
  } else {
    dv = xr[r * NP1 + 1];
  }
  return v + dv;
}

// ---------------------------------------------------------------------------
// Shared memory of one instance (N=16: 40.8 KB -> 4 instances per CU).

template <int N>
struct Smem {
  double Ab[126 * N - 18];  // scaled constraint values, CSC order
  double Gm[N][144];        // G_k (12x12 row-major); during factorisation Q_k [0,36) and
                            // P+sigma of the states [36,48); in the prologue xref/fsteps/gait
  union {
    struct {
      double bd[N][12];  // dynamics-row exchange
      double be[N][8];   // beta exchange
      double ws[N][12];  // bt -> y (forward recurrence)
      double xs[N][12];  // w -> X (backward recurrence)
    } it;
    struct {
      double Lm[144], Sp[144], Gt[144], Dm[144];
    } fa;
  } u;
  unsigned char rc[44 * N];  // constraint class per row (stage ordered)
  int flag[4];
};

// prologue aliases inside Gm
template <int N>
struct Prologue {
  static constexpr int XR = 0;                 // xref, 12(N+1) doubles
  static constexpr int FS = 12 * (N + 1);      // fsteps, 260 doubles
  static constexpr int INTS = FS + 260;        // phase_of_stage[N], contact[20][4] as ints
};

// ---------------------------------------------------------------------------
// scaled-A accessors (stage k)
template <int N>
struct AV {
  const double* Ab;
  // dynamics row i (6..11) of stage k on force column a = 3f + c
  __device__ __forceinline__ double B(int k, int i, int f, int c) const {
    if (i <= 8) return (c == i - 6) ? Ab[FO<N>(k, f, c)] : 0.0;
    return Ab[FO<N>(k, f, c) + i - 8];
  }
  __device__ __forceinline__ double Xd(int k, int i) const { return Ab[XO<N>(k, i)]; }
  // dynamics row i of stage k on X^{k-1}[i] (k >= 1)
  __device__ __forceinline__ double Hd(int k, int i) const {
    return Ab[XO<N>(k - 1, i) + (i < 6 ? 1 : 2)];
  }
  // dynamics row i (< 6) of stage k on X^{k-1}[i+6] (k >= 1)
  __device__ __forceinline__ double H6(int k, int i) const { return Ab[XO<N>(k - 1, i + 6) + 1]; }
  __device__ __forceinline__ double Sw(int k, int f, int c) const { return Ab[FO<N>(k, f, c) + 4]; }
  // friction row 5f+t on component c (0 when absent)
  __device__ __forceinline__ double Fr(int k, int f, int t, int c) const {
    int off = -1;
    if (c == 0 && t < 2) off = 5 + t;
    else if (c == 1 && (t == 2 || t == 3)) off = 5 + (t - 2);
    else if (c == 2) off = 5 + t;
    return off >= 0 ? Ab[FO<N>(k, f, c) + off] : 0.0;
  }
};

struct Rho {
  double v[5];
  __device__ __forceinline__ double operator()(int cls) const {
    return cls == RC_INEQ ? v[1] : (cls == RC_EQ ? v[2] : (cls == RC_LOOSE ? v[0] : (cls == RC_POL_ACT ? v[3] : v[4])));
  }
};

// ---------------------------------------------------------------------------
// The engine kernel.  FUSED: formulate from (xref, fsteps) then solve.
// !FUSED: solve the given (Ax, l, u).  SOLVE=false: formulation only.

template <int N, bool FUSED, bool SOLVE>
__global__ __launch_bounds__(64 * (N / 16), 1) void engine_kernel(mpcq_params p, LaunchArgs a) {
  constexpr int NW = N / 16, T = 64 * NW, n = 24 * N, m = 44 * N, nnz = 126 * N - 18;
  __shared__ Smem<N> sh;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int k = t >> 2, q = t & 3;
  const int64_t b = blockIdx.x;
  if (b >= a.batch) return;
  STAMP_DECL
  const AV<N> A{sh.Ab};
  double* const gm0 = &sh.Gm[0][0];

  // own rows: j < 3 dyn 3q+j, j < 6 swing 3q+j-3, else friction 5q+j-6 (stage-local index)
  auto row_i = [&](int j) __attribute__((always_inline)) {
    return j < 3 ? 3 * q + j : (j < 6 ? 12 + 3 * q + (j - 3) : 24 + 5 * q + (j - 6));
  };
  auto nat_row = [&](int j) __attribute__((always_inline)) {
    return j < 3 ? 12 * k + 3 * q + j
                 : (j < 6 ? 12 * N + 12 * k + 3 * q + (j - 3) : 24 * N + 20 * k + 5 * q + (j - 6));
  };
  // own cols: j < 3 force 3q+j, else state 3q+j-3
  auto nat_col = [&](int j) __attribute__((always_inline)) {
    return j < 3 ? 12 * N + 12 * k + 3 * q + j : 12 * k + 3 * q + (j - 3);
  };
  // P diagonal of own column j (MPC.py:255-275)
  auto P0 = [&](int j) __attribute__((always_inline)) -> double {
    if (j < 3) return p.force_weight;
    const int e = j - 3;
    return q == 0 ? p.state_weights[e]
                  : (q == 1 ? p.state_weights[3 + e] : (q == 2 ? p.state_weights[6 + e] : p.state_weights[9 + e]));
  };

  // Bounds.  FUSED: dynamics rows keep one value (l = u, MPC.py:410); swing rows
  // are 0 = 0; friction rows u = 0, l = -inf (-OSQP_INFTY) or -fz_max.  !FUSED:
  // the caller's l / u for every own row.
  double bnd[3];
  double lo_g[FUSED ? 1 : 11], hi_g[FUSED ? 1 : 11];
  if (t == 0) { sh.flag[0] = 0; sh.flag[1] = 0; sh.flag[2] = 0; sh.flag[3] = 0; }

  // ---------------------------------------------------------------- prologue
  if (FUSED || !SOLVE) {
    double* xr = gm0 + Prologue<N>::XR;
    double* fs = gm0 + Prologue<N>::FS;
    int* pos_ = (int*)(gm0 + Prologue<N>::INTS);  // phase_of_stage[N]
    int* con_ = pos_ + N;                         // contact[20][4]
    const double* gx = a.xref + b * 12 * (N + 1);
    const double* gf = a.fsteps + b * 260;
    for (int e = t; e < 12 * (N + 1); e += T) xr[e] = gx[e];
    for (int e = t; e < 260; e += T) fs[e] = gf[e];
    sync_all<NW>();
    if (t == 0) {  // construct_gait + phase walk (MPC.py:635-652, 336-352, 626-631)
      int idx = -1;
      for (int j = 0; j < 20; ++j)
        if (fs[13 * j] == 0.0) { idx = j; break; }
      int bad = idx < 0, kk = 0;
      for (int j = 0; j < (idx < 0 ? 0 : idx) && !bad; ++j) {
        const double d = fs[13 * j];
        if (!(fabs(d) < 1e6)) { bad = 1; break; }
        const int di = (int)d;
        if (di < 0) { bad = 1; break; }
        for (int f = 0; f < 4; ++f) {
          const double xv = fs[13 * j + 1 + 3 * f];
          con_[4 * j + f] = !(isnan(xv) || xv == 0.0);
        }
        for (int s = 0; s < di; ++s, ++kk)
          if (kk < N) pos_[kk] = j;
      }
      if (kk != N) bad = 1;
      sh.flag[0] = bad ? MPCQ_STATUS_BAD_GAIT : 0;
    }
    sync_all<NW>();
    if (sh.flag[0] == 0) {
      for (int c = t; c < 12 * N; c += T) {  // state columns: -I / A (MPC.py:107-115)
        const int kk = c / 12, i = c % 12, xo = XO<N>(kk, i);
        sh.Ab[xo] = -1.0;
        if (kk < N - 1) {
          if (i >= 6) { sh.Ab[xo + 1] = p.dt; sh.Ab[xo + 2] = 1.0; }
          else sh.Ab[xo + 1] = 1.0;
        }
      }
      {  // foot q of stage k
        const int j = pos_[k];
        double lv[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          double ft;
          if (a.mode == MPCQ_MODE_SETUP)
            ft = q == 0 ? p.footholds[4 * r] : (q == 1 ? p.footholds[4 * r + 1]
                                              : (q == 2 ? p.footholds[4 * r + 2] : p.footholds[4 * r + 3]));
          else {
            ft = fs[13 * j + 1 + 3 * q + r];
            if (isnan(ft)) ft = 0.0;  // MPC.py:327
          }
          lv[r] = ft - xr[r * (N + 1) + k];
        }
        form_foot(p, xr[5 * (N + 1) + k], lv[0], lv[1], lv[2], 1.0 - (double)con_[4 * j + q],
                  sh.Ab + FO<N>(k, q, 0));
      }
#pragma unroll
      for (int e = 0; e < 3; ++e) bnd[e] = dyn_bound<N>(p, xr, k, 3 * q + e);
    }
    if (!SOLVE) {
      sync_all<NW>();
      if (t == 0 && a.status) a.status[b] = sh.flag[0];
      if (sh.flag[0] != 0) return;
      double* go = a.Ax_out + b * nnz;
      for (int e = t; e < nnz; e += T) go[e] = sh.Ab[e];
#pragma unroll
      for (int j = 0; j < 11; ++j) {
        double l, u;
        if (j < 3) { l = bnd[j]; u = bnd[j]; }
        else if (j < 6) { l = 0.0; u = 0.0; }
        else { u = 0.0; l = (j == 10) ? -p.fz_max : -INFINITY; }  // l[24N+4::5] = -25 (MPC.py:228)
        a.l_out[b * m + nat_row(j)] = l;
        a.u_out[b * m + nat_row(j)] = u;
      }
      return;
    }
  } else {
    const double* ga = a.Ax + b * nnz;
    for (int e = t; e < nnz; e += T) sh.Ab[e] = ga[e];
    if constexpr (!FUSED) {
#pragma unroll
      for (int j = 0; j < 11; ++j) {
        lo_g[j] = a.l[b * m + nat_row(j)];
        hi_g[j] = a.u[b * m + nat_row(j)];
      }
    }
  }
  if constexpr (SOLVE) {
    sync_all<NW>();
    int status = sh.flag[0];
    {  // non-finite data -> NONFINITE (the problem is always feasible otherwise)
      int bad = 0;
      for (int e = t; e < nnz; e += T)
        if (!isfinite(sh.Ab[e])) bad = 1;
      if constexpr (FUSED) {
#pragma unroll
        for (int e = 0; e < 3; ++e) if (isnan(bnd[e])) bad = 1;
      } else {
#pragma unroll
        for (int j = 0; j < 11; ++j) {
          if (isnan(lo_g[j]) || isnan(hi_g[j])) bad = 1;
          lo_g[j] = lo_g[j] < -kInf ? -kInf : lo_g[j];  // python osqp clamps to +-OSQP_INFTY
          hi_g[j] = hi_g[j] > kInf ? kInf : hi_g[j];
        }
      }
      if (status == 0 && bad) atomicOr(&sh.flag[1], 1);
      sync_all<NW>();
      if (status == 0 && sh.flag[1]) status = MPCQ_STATUS_NONFINITE;
    }

    // persistent per-lane state: columns [0,3) forces 3q.., [3,6) states 3q..
    double x[6], D[6];
    double z[11], y[11], E[11];
    double Fr[3][12], Sr[3][12];
    unsigned int cpack0 = 0u, cpack1 = 0u;  // constraint class per own row, 3 bits each
#pragma unroll
    for (int j = 0; j < 6; ++j) { x[j] = 0.0; D[j] = 1.0; }
#pragma unroll
    for (int j = 0; j < 11; ++j) { z[j] = 0.0; y[j] = 0.0; E[j] = 1.0; }
#pragma unroll
    for (int e = 0; e < 3; ++e)
#pragma unroll
      for (int j = 0; j < 12; ++j) { Fr[e][j] = 0.0; Sr[e][j] = 0.0; }
    double cscale = 1.0;
    int it_done = 0, n_upd = 0;
    double rho_s = a.rho_in ? a.rho_in[b] : p.rho;
    rho_s = fmin(fmax(rho_s, kRhoMin), kRhoMax);
    Rho rho{{kRhoMin, rho_s, kRhoEq * rho_s, 1.0 / p.delta, 0.0}};
    Rho rinv{{1.0 / kRhoMin, 1.0 / rho_s, 1.0 / (kRhoEq * rho_s), p.delta, 0.0}};

    auto cls = [&](int j) __attribute__((always_inline)) -> int {
      return (int)((j < 10 ? (cpack0 >> (3 * j)) : (cpack1 >> (3 * (j - 10)))) & 7u);
    };
    // scaled bounds of own row j
    auto lo_of = [&](int j) __attribute__((always_inline)) -> double {
      if constexpr (FUSED) {
        if (j < 3) return bnd[j];
        if (j < 6) return 0.0;
        return (j == 10 ? -p.fz_max : -kInf) * E[j];
      } else {
        return lo_g[j];
      }
    };
    auto hi_of = [&](int j) __attribute__((always_inline)) -> double {
      if constexpr (FUSED) {
        if (j < 3) return bnd[j];
        return 0.0;
      } else {
        return hi_g[j];
      }
    };
    auto Pbar = [&](int j) __attribute__((always_inline)) -> double {  // c D P D
      return cscale * (D[j] * P0(j) * D[j]);
    };

    // ---- column / row operators on the stage layout ---------------------
    // A' w for own columns.  wown = w of own rows; dyn-row w of all stages in bd.
    auto col_At = [&](const double (&wown)[11], double (&out)[6]) __attribute__((always_inline)) {
      const double* wk = sh.u.it.bd[k];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int fo = FO<N>(k, q, c);
        double s = sh.Ab[fo] * wk[6 + c];
        s += sh.Ab[fo + 1] * wk[9];
        s += sh.Ab[fo + 2] * wk[10];
        s += sh.Ab[fo + 3] * wk[11];
        s += sh.Ab[fo + 4] * wown[3 + c];
        if (c == 0) { s += sh.Ab[fo + 5] * wown[6]; s += sh.Ab[fo + 6] * wown[7]; }
        else if (c == 1) { s += sh.Ab[fo + 5] * wown[8]; s += sh.Ab[fo + 6] * wown[9]; }
        else {
#pragma unroll
          for (int tt = 0; tt < 5; ++tt) s += sh.Ab[fo + 5 + tt] * wown[6 + tt];
        }
        out[c] = s;
      }
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const int i = 3 * q + e, xo = XO<N>(k, i);
        double s = sh.Ab[xo] * wown[e];
        if (k < N - 1) {
          const double* wn = sh.u.it.bd[k + 1];
          if (i >= 6) { s += sh.Ab[xo + 1] * wn[i - 6]; s += sh.Ab[xo + 2] * wn[i]; }
          else s += sh.Ab[xo + 1] * wn[i];
        }
        out[3 + e] = s;
      }
    };
    // (B f)_{6..11} of the stage from the own force columns (quad sums; all lanes)
    auto Bf6 = [&](const double (&fown)[3], double (&bf6)[6]) __attribute__((always_inline)) {
      double pp[6];
#pragma unroll
      for (int c = 0; c < 3; ++c) pp[c] = sh.Ab[FO<N>(k, q, c)] * fown[c];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < 3; ++c) s += sh.Ab[FO<N>(k, q, c) + 1 + r] * fown[c];
        pp[3 + r] = s;
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) bf6[j] = quad_sum(pp[j]);
    };
    // A v for own rows: fown = own forces, vx = own states, previous stage's states in xs[k-1]
    auto row_A = [&](const double (&fown)[3], const double (&vx)[3], double (&out)[11]) __attribute__((always_inline)) {
      double bf6[6];
      Bf6(fown, bf6);
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const int i = 3 * q + e;
        double s = 0.0;
        if (k >= 1) {
          const double* xp = sh.u.it.xs[k - 1];
          s += A.Hd(k, i) * xp[i];
          if (i < 6) s += A.H6(k, i) * xp[i + 6];
        }
        s += A.Xd(k, i) * vx[e];
        if (q == 2) s += bf6[e];
        else if (q == 3) s += bf6[3 + e];
        out[e] = s;
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) out[3 + c] = A.Sw(k, q, c) * fown[c];
      const int b0 = FO<N>(k, q, 0), b1 = FO<N>(k, q, 1), b2 = FO<N>(k, q, 2);
      out[6] = sh.Ab[b0 + 5] * fown[0] + sh.Ab[b2 + 5] * fown[2];
      out[7] = sh.Ab[b0 + 6] * fown[0] + sh.Ab[b2 + 6] * fown[2];
      out[8] = sh.Ab[b1 + 5] * fown[1] + sh.Ab[b2 + 7] * fown[2];
      out[9] = sh.Ab[b1 + 6] * fown[1] + sh.Ab[b2 + 8] * fown[2];
      out[10] = sh.Ab[b2 + 9] * fown[2];
    };
    // per-row rho of a dynamics row (k', i) from the class table
    auto rho_dyn = [&](int kk, int i) __attribute__((always_inline)) { return rho((int)sh.rc[44 * kk + i]); };

    // ---- factorisation -----------------------------------------------------
    // Phase P (every quad, its stage): F = K_ff^{-1}, Q = W' F W.  Phase S (wave
    // 0, 48 lanes, sequential in k): S_k^{-1}, G_k.
    auto factor = [&](double sigma) __attribute__((always_inline)) -> bool {
      bool ok = true;
      {
        // K_ff rows 3q+c, built in place in Fr and inverted there
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int bb = 0; bb < 12; ++bb) {
            const int fb = bb / 3, cbb = bb % 3;
            double v = 0.0;
#pragma unroll
            for (int i = 6; i < 12; ++i) {
              const double ba = A.B(k, i, q, c), bbv = A.B(k, i, fb, cbb);
              v += rho_dyn(k, i) * ba * bbv;
            }
            if (bb == 3 * q + c) {
              const double sw = A.Sw(k, q, c);
              v += Pbar(c) + sigma + rho(cls(3 + c)) * sw * sw;
            }
            if (fb == q) {
#pragma unroll
              for (int tt = 0; tt < 5; ++tt)
                v += rho(cls(6 + tt)) * A.Fr(k, q, tt, c) * A.Fr(k, q, tt, cbb);
            }
            Fr[c][bb] = v;
          }
        // Gauss-Jordan inverse inside the quad (SPD, no pivoting)
#pragma unroll
        for (int pv = 0; pv < 12; ++pv) {
          const int pl = pv / 3, pe = pv % 3;
          double prow[12];
#pragma unroll
          for (int j = 0; j < 12; ++j) {
            const double src = Fr[pe][j];
            prow[j] = pl == 0 ? qbcast<0>(src) : (pl == 1 ? qbcast<1>(src) : (pl == 2 ? qbcast<2>(src) : qbcast<3>(src)));
          }
          const double d = prow[pv];
          if (!(d > 0.0)) ok = false;
          const double id = 1.0 / d;
#pragma unroll
          for (int e = 0; e < 3; ++e) {
            const bool isp = (q == pl) && (e == pe);
            const double mrp = Fr[e][pv];
#pragma unroll
            for (int j = 0; j < 12; ++j) {
              double v;
              if (isp) v = (j == pv) ? id : prow[j] * id;
              else v = (j == pv) ? -mrp * id : Fr[e][j] - mrp * prow[j] * id;
              Fr[e][j] = v;
            }
          }
        }
        // Q = W' F W (6x6), W[bb][j] = rho_{6+j} B[6+j][bb]; one column of F W at a time
#pragma unroll
        for (int jj = 0; jj < 6; ++jj) {
          double zc[3] = {0.0, 0.0, 0.0};
          const double rj = rho_dyn(k, 6 + jj);
#pragma unroll
          for (int bb = 0; bb < 12; ++bb) {
            const double w = rj * A.B(k, 6 + jj, bb / 3, bb % 3);
#pragma unroll
            for (int e = 0; e < 3; ++e) zc[e] += Fr[e][bb] * w;
          }
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            double s = 0.0;
#pragma unroll
            for (int e = 0; e < 3; ++e) s += rho_dyn(k, 6 + j) * A.B(k, 6 + j, q, e) * zc[e];
            s = quad_sum(s);
            if (q == 0) sh.Gm[k][6 * j + jj] = s;
          }
        }
#pragma unroll
        for (int e = 0; e < 3; ++e) sh.Gm[k][36 + 3 * q + e] = Pbar(3 + e) + sigma;
      }
      sync_all<NW>();
      // Phase S
      const int r = lane >> 2, cb = lane & 3;
      const bool act = (wv == 0) && lane < 48;
      double* Lm = sh.u.fa.Lm;
      double* Sp = sh.u.fa.Sp;
      double* Gt = sh.u.fa.Gt;
      for (int kk = 0; kk < N; ++kk) {
        double mreg[3] = {0.0, 0.0, 0.0};
        if (wv == 0) {
          double Dv[3], Lv[3];
          if (act) {
            const double xdr = A.Xd(kk, r);
            const double* Qk = sh.Gm[kk];
#pragma unroll
            for (int e = 0; e < 3; ++e) {
              const int c = 3 * cb + e;
              double v = 0.0;
              if (r == c) v = sh.Gm[kk][36 + r] + rho_dyn(kk, r) * xdr * xdr;
              if (kk < N - 1) {
                // dynamics rows of stage kk+1 on X^kk (coefficients live in X^kk's columns)
                const double hr = A.Hd(kk + 1, r);
                if (r == c) {
                  v += rho_dyn(kk + 1, r) * hr * hr;
                  if (r >= 6) { const double h6 = A.H6(kk + 1, r - 6); v += rho_dyn(kk + 1, r - 6) * h6 * h6; }
                }
                if (c == r + 6) v += rho_dyn(kk + 1, r) * hr * A.H6(kk + 1, r);
                if (r == c + 6) v += rho_dyn(kk + 1, c) * A.Hd(kk + 1, c) * A.H6(kk + 1, c);
              }
              if (r >= 6 && c >= 6) {
                v -= xdr * Qk[6 * (r - 6) + (c - 6)] * A.Xd(kk, c);
                if (kk < N - 1) v -= A.Hd(kk + 1, r) * sh.Gm[kk + 1][6 * (r - 6) + (c - 6)] * A.Hd(kk + 1, c);
              }
              Dv[e] = v;
              double l = 0.0;
              if (kk >= 1) {
                if (c == r) l = rho_dyn(kk, r) * xdr * A.Hd(kk, r);
                else if (c == r + 6 && r < 6) l = rho_dyn(kk, r) * xdr * A.H6(kk, r);
                if (r >= 6 && c >= 6) l -= xdr * Qk[6 * (r - 6) + (c - 6)] * A.Hd(kk, c);
              }
              Lv[e] = l;
            }
          }
          if (kk >= 1) {
            if (act) {
#pragma unroll
              for (int e = 0; e < 3; ++e) Lm[12 * r + 3 * cb + e] = Lv[e];
            }
            wave_sync();
            double g[3] = {0.0, 0.0, 0.0};
            if (act) {
#pragma unroll
              for (int tt = 0; tt < 12; ++tt) {
                const double lrt = Lm[12 * r + tt];
#pragma unroll
                for (int e = 0; e < 3; ++e) g[e] += lrt * Sp[12 * tt + 3 * cb + e];
              }
#pragma unroll
              for (int e = 0; e < 3; ++e) Gt[12 * r + 3 * cb + e] = g[e];
            }
            wave_sync();
            if (act) {
#pragma unroll
              for (int e = 0; e < 3; ++e) {
                const int c = 3 * cb + e;
                double s = 0.0;
#pragma unroll
                for (int tt = 0; tt < 12; ++tt) s += Gt[12 * r + tt] * Lm[12 * c + tt];
                mreg[e] = Dv[e] - s;
              }
            }
          } else {
#pragma unroll
            for (int e = 0; e < 3; ++e) mreg[e] = act ? Dv[e] : 0.0;
          }
          // Gauss-Jordan inverse of S_kk, entries (r, 3cb..3cb+2), via lane shuffles
#pragma unroll
          for (int pv = 0; pv < 12; ++pv) {
            const int pl = pv / 3, pe = pv % 3;
            const double pr0 = __shfl(mreg[0], 4 * pv + cb);
            const double pr1 = __shfl(mreg[1], 4 * pv + cb);
            const double pr2 = __shfl(mreg[2], 4 * pv + cb);
            const double msel = pe == 0 ? mreg[0] : (pe == 1 ? mreg[1] : mreg[2]);
            const double mcol = __shfl(msel, 4 * r + pl);
            const double d = __shfl(msel, 4 * pv + pl);
            if (!(d > 0.0)) ok = false;
            const double id = 1.0 / d;
            const double prow[3] = {pr0, pr1, pr2};
#pragma unroll
            for (int e = 0; e < 3; ++e) {
              const int c = 3 * cb + e;
              double v;
              if (r == pv) v = (c == pv) ? id : prow[e] * id;
              else v = (c == pv) ? -mcol * id : mreg[e] - mcol * prow[e] * id;
              mreg[e] = v;
            }
          }
          if (act) {
#pragma unroll
            for (int e = 0; e < 3; ++e) Sp[12 * r + 3 * cb + e] = mreg[e];
          }
        }
        sync_all<NW>();
        // G_kk -> Gm[kk] (the Q / P entries of stage kk are no longer needed)
        if (act) {
#pragma unroll
          for (int e = 0; e < 3; ++e) sh.Gm[kk][12 * r + 3 * cb + e] = (kk >= 1) ? Gt[12 * r + 3 * cb + e] : 0.0;
        }
        if (k == kk) {
#pragma unroll
          for (int e = 0; e < 3; ++e)
#pragma unroll
            for (int j = 0; j < 12; ++j) Sr[e][j] = Sp[12 * (3 * q + e) + j];
        }
        sync_all<NW>();
      }
      // a non-positive pivot anywhere fails the whole instance (uniform result)
      if (!ok) atomicOr(&sh.flag[2], 1);
      sync_all<NW>();
      const bool good = sh.flag[2] == 0;
      sync_all<NW>();
      return good;
    };

    // ---- KKT solve: (bf, bX) own columns -> (sf, sX) own columns ----------
    auto kkt_solve = [&](const double (&bf)[3], const double (&bX)[3], double (&sf)[3],
                         double (&sX)[3]) __attribute__((always_inline)) {
      double ball[12], u[3];
      quad_gather12(bf, ball);
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < 12; ++j) s += Fr[e][j] * ball[j];
        u[e] = s;
      }
      double bu6[6];
      Bf6(u, bu6);  // beta = rho (B u)_{6..11}
      if (q == 0) {
#pragma unroll
        for (int j = 0; j < 6; ++j) sh.u.it.be[k][j] = rho_dyn(k, 6 + j) * bu6[j];
      }
      // bt_X without the next stage's beta term (the recurrence adds it)
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const int i = 3 * q + e;
        double bt = bX[e];
        if (q >= 2) {
          const double bown = rho_dyn(k, i) * (q == 2 ? bu6[e] : bu6[3 + e]);
          bt -= A.Xd(k, i) * bown;
        }
        sh.u.it.ws[k][i] = bt;
      }
      sync_all<NW>();
      STAMP(4);
      // forward recurrence y_k = bt_k - Hd_{k+1} beta_{k+1} - G_k y_{k-1} (wave 0, lane (r, cb))
      if (wv == 0) {
        const int r = lane >> 2, cb = lane & 3;
        const bool act = lane < 48;
        double p0 = 0.0, p1 = 0.0, p2 = 0.0;
        for (int kk = 0; kk < N; ++kk) {
          double g0 = 0.0, g1 = 0.0, g2 = 0.0, bt = 0.0;
          if (act) {
            const double* G = sh.Gm[kk] + 12 * r + 3 * cb;
            g0 = G[0]; g1 = G[1]; g2 = G[2];
            bt = sh.u.it.ws[kk][r];
            if (r >= 6 && kk < N - 1) bt -= A.Hd(kk + 1, r) * sh.u.it.be[kk + 1][r - 6];
          }
          double acc = g0 * p0 + g1 * p1 + g2 * p2;
          acc = quad_sum(acc);
          const double yr = bt - acc;
          if (act && cb == 0) sh.u.it.ws[kk][r] = yr;
          p0 = __shfl(yr, 4 * (3 * cb + 0));
          p1 = __shfl(yr, 4 * (3 * cb + 1));
          p2 = __shfl(yr, 4 * (3 * cb + 2));
        }
      }
      sync_all<NW>();
      STAMP(5);
      // w_k = S_k^{-1} y_k
      {
        double yall[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) yall[j] = sh.u.it.ws[k][j];
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          double s = 0.0;
#pragma unroll
          for (int j = 0; j < 12; ++j) s += Sr[e][j] * yall[j];
          sh.u.it.xs[k][3 * q + e] = s;
        }
      }
      sync_all<NW>();
      STAMP(6);
      // backward recurrence X_k = w_k - G_{k+1}' X_{k+1}
      if (wv == 0) {
        const int r = lane >> 2, cb = lane & 3;
        const bool act = lane < 48;
        double p0 = 0.0, p1 = 0.0, p2 = 0.0;
        for (int kk = N - 1; kk >= 0; --kk) {
          double g0 = 0.0, g1 = 0.0, g2 = 0.0, w = 0.0;
          if (act) {
            w = sh.u.it.xs[kk][r];
            if (kk < N - 1) {
              const double* G = sh.Gm[kk + 1] + r;
              g0 = G[12 * (3 * cb + 0)]; g1 = G[12 * (3 * cb + 1)]; g2 = G[12 * (3 * cb + 2)];
            }
          }
          double acc = g0 * p0 + g1 * p1 + g2 * p2;
          acc = quad_sum(acc);
          const double xr = w - acc;
          if (act && cb == 0) sh.u.it.xs[kk][r] = xr;
          p0 = __shfl(xr, 4 * (3 * cb + 0));
          p1 = __shfl(xr, 4 * (3 * cb + 1));
          p2 = __shfl(xr, 4 * (3 * cb + 2));
        }
      }
      sync_all<NW>();
      STAMP(7);
      // forces: f_k = F_k (b_f - W_k gamma_k)
      double gam[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int i = 6 + j;
        double g = A.Xd(k, i) * sh.u.it.xs[k][i];
        if (k >= 1) g += A.Hd(k, i) * sh.u.it.xs[k - 1][i];
        gam[j] = rho_dyn(k, i) * g;
      }
      double rf[3], rall[12];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int fo = FO<N>(k, q, c);
        double wg = sh.Ab[fo] * gam[c];
        wg += sh.Ab[fo + 1] * gam[3];
        wg += sh.Ab[fo + 2] * gam[4];
        wg += sh.Ab[fo + 3] * gam[5];
        rf[c] = bf[c] - wg;
      }
      quad_gather12(rf, rall);
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < 12; ++j) s += Fr[e][j] * rall[j];
        sf[e] = s;
        sX[e] = sh.u.it.xs[k][3 * q + e];
      }
    };

    // ---- residuals (OSQP update_info), uniform results ---------------------
    double pri_res = 0.0, dua_res = 0.0, eps_pri = 0.0, eps_dua = 0.0, s_pri = 0.0, s_dua = 0.0;
    auto update_info = [&]() __attribute__((always_inline)) {
      sync_all<NW>();
#pragma unroll
      for (int e = 0; e < 3; ++e) { sh.u.it.xs[k][3 * q + e] = x[3 + e]; sh.u.it.bd[k][3 * q + e] = y[e]; }
      sync_all<NW>();
      double qv[12];
#pragma unroll
      for (int e = 0; e < 12; ++e) qv[e] = 0.0;
      {
        const double xf[3] = {x[0], x[1], x[2]}, xX[3] = {x[3], x[4], x[5]};
        double ax[11];
        row_A(xf, xX, ax);
#pragma unroll
        for (int j = 0; j < 11; ++j) {
          const double ei = 1.0 / E[j], d = ax[j] - z[j];
          qv[0] = fmax(qv[0], fabs(ei * d));
          qv[1] = fmax(qv[1], fabs(ei * ax[j]));
          qv[2] = fmax(qv[2], fabs(ei * z[j]));
          qv[3] = fmax(qv[3], fabs(d));
          qv[4] = fmax(qv[4], fabs(ax[j]));
          qv[5] = fmax(qv[5], fabs(z[j]));
        }
      }
      {
        double aty[6];
        col_At(y, aty);
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          const double px = Pbar(j) * x[j], di = 1.0 / D[j], d = px + 0.0 + aty[j];
          qv[6] = fmax(qv[6], fabs(di * d));
          qv[7] = fmax(qv[7], fabs(di * px));
          qv[8] = fmax(qv[8], fabs(di * aty[j]));
          qv[9] = fmax(qv[9], fabs(d));
          qv[10] = fmax(qv[10], fabs(px));
          qv[11] = fmax(qv[11], fabs(aty[j]));
        }
      }
#pragma unroll
      for (int e = 0; e < 12; ++e) qv[e] = wave_max(qv[e]);
      if constexpr (NW > 1) {
        sync_all<NW>();
        double* red = &sh.u.it.ws[0][0];
        if (lane == 0) {
#pragma unroll
          for (int e = 0; e < 12; ++e) red[16 * wv + e] = qv[e];
        }
        sync_all<NW>();
#pragma unroll
        for (int e = 0; e < 12; ++e) {
          double v = 0.0;
#pragma unroll
          for (int w = 0; w < NW; ++w) v = fmax(v, red[16 * w + e]);
          qv[e] = v;
        }
      }
      const double cinv = 1.0 / cscale;
      pri_res = qv[0];
      dua_res = cinv * qv[6];
      eps_pri = p.eps_abs + p.eps_rel * fmax(qv[1], qv[2]);
      eps_dua = p.eps_abs + p.eps_rel * cinv * fmax(qv[7], qv[8]);
      s_pri = qv[3] / (fmax(qv[4], qv[5]) + kDivTol);
      s_dua = qv[9] / (fmax(qv[10], qv[11]) + kDivTol);
      sync_all<NW>();
    };
    auto converged = [&](double f) __attribute__((always_inline)) {
      return pri_res < f * eps_pri && dua_res < f * eps_dua;
    };

    if (status == 0) {
      STAMP(0);
      // ------------------------------------------------------------ Ruiz scaling
      {
        double Pb[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) Pb[j] = P0(j);
        for (int it = 0; it < p.scaling; ++it) {
          double dtv[6], etv[11];
#pragma unroll
          for (int c = 0; c < 3; ++c) {  // column norms of [P; A]
            const int fo = FO<N>(k, q, c);
            const int cnt = c < 2 ? 7 : 10;
            double v = fabs(Pb[c]);
            for (int e = 0; e < cnt; ++e) v = fmax(v, fabs(sh.Ab[fo + e]));
            dtv[c] = v;
          }
#pragma unroll
          for (int e = 0; e < 3; ++e) {
            const int i = 3 * q + e, xo = XO<N>(k, i);
            const int cnt = (k < N - 1) ? (i < 6 ? 2 : 3) : 1;
            double v = fabs(Pb[3 + e]);
            for (int h = 0; h < cnt; ++h) v = fmax(v, fabs(sh.Ab[xo + h]));
            dtv[3 + e] = v;
          }
#pragma unroll
          for (int e = 0; e < 3; ++e) {  // row norms of A
            const int i = 3 * q + e;
            double v = fabs(A.Xd(k, i));
            if (k >= 1) {
              v = fmax(v, fabs(A.Hd(k, i)));
              if (i < 6) v = fmax(v, fabs(A.H6(k, i)));
            }
            if (q == 2) {
#pragma unroll
              for (int f = 0; f < 4; ++f) v = fmax(v, fabs(sh.Ab[FO<N>(k, f, e)]));
            } else if (q == 3) {
#pragma unroll
              for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int c = 0; c < 3; ++c) v = fmax(v, fabs(sh.Ab[FO<N>(k, f, c) + 1 + e]));
            }
            etv[e] = v;
          }
#pragma unroll
          for (int c = 0; c < 3; ++c) etv[3 + c] = fabs(A.Sw(k, q, c));
          {
            const int b0 = FO<N>(k, q, 0), b1 = FO<N>(k, q, 1), b2 = FO<N>(k, q, 2);
            etv[6] = fmax(fabs(sh.Ab[b0 + 5]), fabs(sh.Ab[b2 + 5]));
            etv[7] = fmax(fabs(sh.Ab[b0 + 6]), fabs(sh.Ab[b2 + 6]));
            etv[8] = fmax(fabs(sh.Ab[b1 + 5]), fabs(sh.Ab[b2 + 7]));
            etv[9] = fmax(fabs(sh.Ab[b1 + 6]), fabs(sh.Ab[b2 + 8]));
            etv[10] = fabs(sh.Ab[b2 + 9]);
          }
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            double v = dtv[j];
            v = v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v);
            dtv[j] = 1.0 / sqrt(v);
            D[j] *= dtv[j];
            Pb[j] = dtv[j] * Pb[j] * dtv[j];
          }
#pragma unroll
          for (int j = 0; j < 11; ++j) {
            double v = etv[j];
            v = v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v);
            etv[j] = 1.0 / sqrt(v);
            E[j] *= etv[j];
          }
          // exchange the dyn-row factors; scale own columns' entries (E_r A D_c)
#pragma unroll
          for (int e = 0; e < 3; ++e) sh.u.it.bd[k][3 * q + e] = etv[e];
          sync_all<NW>();
          {
            const double* ek = sh.u.it.bd[k];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const int fo = FO<N>(k, q, c);
              const double dt = dtv[c];
              sh.Ab[fo] = ek[6 + c] * sh.Ab[fo] * dt;
              sh.Ab[fo + 1] = ek[9] * sh.Ab[fo + 1] * dt;
              sh.Ab[fo + 2] = ek[10] * sh.Ab[fo + 2] * dt;
              sh.Ab[fo + 3] = ek[11] * sh.Ab[fo + 3] * dt;
              sh.Ab[fo + 4] = etv[3 + c] * sh.Ab[fo + 4] * dt;
              if (c == 0) { sh.Ab[fo + 5] = etv[6] * sh.Ab[fo + 5] * dt; sh.Ab[fo + 6] = etv[7] * sh.Ab[fo + 6] * dt; }
              else if (c == 1) { sh.Ab[fo + 5] = etv[8] * sh.Ab[fo + 5] * dt; sh.Ab[fo + 6] = etv[9] * sh.Ab[fo + 6] * dt; }
              else {
#pragma unroll
                for (int tt = 0; tt < 5; ++tt) sh.Ab[fo + 5 + tt] = etv[6 + tt] * sh.Ab[fo + 5 + tt] * dt;
              }
            }
#pragma unroll
            for (int e = 0; e < 3; ++e) {
              const int i = 3 * q + e, xo = XO<N>(k, i);
              const double dt = dtv[3 + e];
              sh.Ab[xo] = etv[e] * sh.Ab[xo] * dt;
              if (k < N - 1) {
                const double* en = sh.u.it.bd[k + 1];
                if (i >= 6) {
                  sh.Ab[xo + 1] = en[i - 6] * sh.Ab[xo + 1] * dt;
                  sh.Ab[xo + 2] = en[i] * sh.Ab[xo + 2] * dt;
                } else {
                  sh.Ab[xo + 1] = en[i] * sh.Ab[xo + 1] * dt;
                }
              }
            }
          }
          // cost scaling: c = 1 / max(mean |P|, 1)  (q = 0)
          double ps = 0.0;
#pragma unroll
          for (int j = 0; j < 6; ++j) ps += fabs(Pb[j]);
          ps = wave_sum(ps);
          if constexpr (NW > 1) {
            double* red = sh.u.it.ws[0];
            sync_all<NW>();
            if (lane == 0) red[wv] = ps;
            sync_all<NW>();
            ps = 0.0;
#pragma unroll
            for (int w = 0; w < NW; ++w) ps += red[w];
          }
          const double mean = ps / n;
          double ctmp = mean > 1.0 ? mean : 1.0;
          ctmp = ctmp < kMinScaling ? 1.0 : (ctmp > kMaxScaling ? kMaxScaling : ctmp);
          ctmp = 1.0 / ctmp;
#pragma unroll
          for (int j = 0; j < 6; ++j) Pb[j] *= ctmp;
          cscale *= ctmp;
          sync_all<NW>();
        }
      }
      // scaled bounds, constraint classes (osqp set_rho_vec)
      if constexpr (FUSED) {
#pragma unroll
        for (int e = 0; e < 3; ++e) bnd[e] *= E[e];
      } else {
#pragma unroll
        for (int j = 0; j < 11; ++j) { lo_g[j] *= E[j]; hi_g[j] *= E[j]; }
      }
#pragma unroll
      for (int j = 0; j < 11; ++j) {
        const double lj = lo_of(j), hj = hi_of(j);
        unsigned int c;
        if (lj < -kInf * kMinScaling && hj > kInf * kMinScaling) c = RC_LOOSE;
        else if (hj - lj < kRhoTol) c = RC_EQ;
        else c = RC_INEQ;
        if (j < 10) cpack0 |= c << (3 * j);
        else cpack1 |= c << (3 * (j - 10));
        sh.rc[44 * k + row_i(j)] = (unsigned char)c;
      }
      // warm start (osqp_warm_start: x = D^-1 x0, z = A x; y = c E^-1 y0)
      if (a.warm_x) {
#pragma unroll
        for (int j = 0; j < 6; ++j) x[j] = a.warm_x[b * n + nat_col(j)] / D[j];
#pragma unroll
        for (int e = 0; e < 3; ++e) sh.u.it.xs[k][3 * q + e] = x[3 + e];
        sync_all<NW>();
        const double xf[3] = {x[0], x[1], x[2]}, xX[3] = {x[3], x[4], x[5]};
        row_A(xf, xX, z);
        sync_all<NW>();
      }
      if (a.warm_y) {
#pragma unroll
        for (int j = 0; j < 11; ++j) y[j] = cscale * a.warm_y[b * m + nat_row(j)] / E[j];
      }
      sync_all<NW>();
      STAMP(1);

      // ------------------------------------------------------------ ADMM
      // The factorisation sits outside the hot loop: the outer loop factors,
      // the inner loop iterates until convergence, max_iter or a rho update.
      bool last_checked = false;
      int iter = 1;
      for (;;) {
        if (!factor(p.sigma)) { status = MPCQ_STATUS_FACTOR_FAILED; break; }
        STAMP(2);
        bool refactor = false;
        for (; iter <= p.max_iter; ++iter) {
          // w = rho z - y (own rows); dyn rows exchanged through LDS
          double w[11];
#pragma unroll
          for (int j = 0; j < 11; ++j) w[j] = rho(cls(j)) * z[j] - y[j];
#pragma unroll
          for (int e = 0; e < 3; ++e) sh.u.it.bd[k][3 * q + e] = w[e];
          sync_all<NW>();
          STAMP(3);
          double bf[3], bX[3];
          {
            double bv[6];
            col_At(w, bv);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              bf[j] = bv[j] + p.sigma * x[j];  // - q, q = 0
              bX[j] = bv[3 + j] + p.sigma * x[3 + j];
            }
          }
          double sf[3], sX[3];
          kkt_solve(bf, bX, sf, sX);
          STAMP(8);
          // z, y update (osqp update_z / update_y), x update
          {
            double ax[11];
            row_A(sf, sX, ax);
#pragma unroll
            for (int j = 0; j < 11; ++j) {
              const int cj = cls(j);
              const double zr = p.alpha * ax[j] + (1.0 - p.alpha) * z[j];
              const double tt = zr + rinv(cj) * y[j];
              const double lj = lo_of(j), hj = hi_of(j);
              const double zn = tt < lj ? lj : (tt > hj ? hj : tt);
              y[j] = y[j] + rho(cj) * (zr - zn);
              z[j] = zn;
            }
          }
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            x[j] = p.alpha * sf[j] + (1.0 - p.alpha) * x[j];
            x[3 + j] = p.alpha * sX[j] + (1.0 - p.alpha) * x[3 + j];
          }
          STAMP(9);
          const bool can_check = p.check_termination > 0 && (iter % p.check_termination == 0);
          const bool adapt = p.adaptive_rho && p.adaptive_rho_interval > 0 &&
                             (iter % p.adaptive_rho_interval == 0);
          last_checked = can_check;
          if (can_check || adapt) {
            update_info();
            if (!(isfinite(pri_res) && isfinite(dua_res))) { status = MPCQ_STATUS_NONFINITE; break; }
            if (can_check && converged(1.0)) { status = MPCQ_STATUS_SOLVED; break; }
            if (adapt) {
              double rn = rho_s * sqrt(s_pri / (s_dua + kDivTol));
              rn = fmin(fmax(rn, kRhoMin), kRhoMax);
              if (rn > rho_s * p.adaptive_rho_tolerance || rn < rho_s / p.adaptive_rho_tolerance) {
                rho_s = rn;
                rho.v[1] = rho_s;
                rho.v[2] = kRhoEq * rho_s;
                rinv.v[1] = 1.0 / rho.v[1];
                rinv.v[2] = 1.0 / rho.v[2];
                refactor = true;
                ++n_upd;
                ++iter;
                sync_all<NW>();
                break;
              }
            }
          }
          sync_all<NW>();
          STAMP(10);
        }
        if (!refactor) break;
      }
      it_done = iter > p.max_iter ? p.max_iter : iter;
      if (status == 0) {
        if (!last_checked) {
          update_info();
          if (converged(1.0)) status = MPCQ_STATUS_SOLVED;
        }
        if (status == 0)
          status = converged(10.0) ? MPCQ_STATUS_SOLVED_INACCURATE : MPCQ_STATUS_MAX_ITER_REACHED;
      }
    }
    // ------------------------------------------------------------ outputs
    const bool nan_out = status == MPCQ_STATUS_NONFINITE || status == MPCQ_STATUS_FACTOR_FAILED ||
                         status == MPCQ_STATUS_BAD_GAIT;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const double xv = nan_out ? NAN : D[j] * x[j];
      if (a.x) a.x[b * n + nat_col(j)] = xv;
      if (a.f0 && k == 0 && j < 3) a.f0[b * 12 + 3 * q + j] = xv;
    }
    if (a.y) {
#pragma unroll
      for (int j = 0; j < 11; ++j) a.y[b * m + nat_row(j)] = nan_out ? NAN : E[j] * y[j] / cscale;
    }
#ifdef MPCQ_STAMPS
    STAMP(11);
    if (t == 0 && a.stamps) {
      for (int i = 0; i < 16; ++i) a.stamps[b * 16 + i] = st_acc[i];
    }
#endif
    if (t == 0) {
      if (a.status) a.status[b] = status;
      if (a.iters) a.iters[b] = it_done;
      if (a.rho_out) a.rho_out[b] = rho_s;
      if (a.info) {
        a.info[4 * b + 0] = n_upd;
        a.info[4 * b + 1] = 0;
        a.info[4 * b + 2] = 0;
        a.info[4 * b + 3] = 0;
      }
    }
  }
}

template <int N>
hipError_t launch_t(bool fused, bool solve, const mpcq_params& p, const LaunchArgs& a,
                    hipStream_t s) {
  const dim3 grid((unsigned)a.batch), block(64 * (N / 16));
  if (!solve) hipLaunchKernelGGL((engine_kernel<N, true, false>), grid, block, 0, s, p, a);
  else if (fused) hipLaunchKernelGGL((engine_kernel<N, true, true>), grid, block, 0, s, p, a);
  else hipLaunchKernelGGL((engine_kernel<N, false, true>), grid, block, 0, s, p, a);
  return hipGetLastError();
}

}  // namespace

bool horizon_supported(int N) { return N == 16 || N == 32; }

int supported_horizons(int32_t* out, int cap) {
  const int32_t hs[2] = {16, 32};
  for (int i = 0; i < 2 && i < cap; ++i) out[i] = hs[i];
  return 2;
}

hipError_t launch_formulate(int N, const mpcq_params& p, const LaunchArgs& a, hipStream_t s) {
  if (a.batch <= 0) return hipSuccess;
  if (N == 16) return launch_t<16>(true, false, p, a, s);
  if (N == 32) return launch_t<32>(true, false, p, a, s);
  return hipErrorInvalidValue;
}

hipError_t launch_solve(int N, bool fused, const mpcq_params& p, const LaunchArgs& a,
                        hipStream_t s) {
  if (a.batch <= 0) return hipSuccess;
  if (N == 16) return launch_t<16>(fused, true, p, a, s);
  if (N == 32) return launch_t<32>(fused, true, p, a, s);
  return hipErrorInvalidValue;
}

}  // namespace mpcq
