// mpcq_kernels.hip — batched convex-MPC QP engine for MI355X (gfx950, CDNA4).
//
// One workgroup owns one QP instance for its whole life: formulation
// (MPC.py:98-378), Ruiz scaling, block-tridiagonal KKT factorisation and the
// OSQP-0.6 ADMM iterations run out of LDS + registers; HBM sees only the
// compulsory inputs (xref, fsteps) and outputs (f0 / x / y / status).
//
// Work split inside the workgroup (NW = N/4 waves of 64 lanes, T = 16N threads):
//   stage k = [f_k (12 forces), X_{k+1} (12 states)] is owned by wave k % NW
//   (slot s = k / NW, 4 slots per wave).  The owner wave keeps
//   S_k^{-1} (24x24 inverse Schur complement of the KKT) in REGISTERS: lane
//   l < 48 holds row l>>1, columns 12*(l&1) .. +11 (12 doubles per stage).
//   Rows (44 per stage: 12 dynamics, 12 swing mask, 20 friction) and columns
//   (24 per stage) of the owner's stages are spread over its 64 lanes; their
//   ADMM vectors (x, z, y, bounds, scaling, rho) live in registers too.
//   LDS holds the scaled constraint values (CSC order, nnz = 126N-18), the
//   12x12 recurrence matrices Gamma_k, and exchange vectors.
//
// KKT solve (P + sigma I + A' R A) w = b, block tridiagonal in stages:
//   S_0 = K_0,  S_k = K_k - C_k Y_{k-1} C_k',  Y = (S^{-1})_XX,  C_k = 24x12
//   forward:  s_k = alpha_k - Gamma_k s_{k-1},  alpha_k = (S_k^{-1})_{X,:} b_k,
//             Gamma_k = (S_k^{-1})_{X,:} C_k              (12x12, sequential)
//             t_k = S_k^{-1} (b_k - C_k s_{k-1})           (parallel over k)
//   backward: v_{k-1} = beta_k - Gamma_k' v_k, beta_k = C_k' t_k (12x12, sequential)
//             w_k = t_k - (S_k^{-1})_{:,X} v_k             (parallel over k)
// Only the two 12-wide recurrences are sequential in k; every 24x24 product
// runs for all stages at once.
#include <math.h>

#include "mpcq_internal.h"

namespace mpcq {
namespace {

constexpr double kInf = 1e30;  // OSQP_INFTY
constexpr double kMinScaling = 1e-4, kMaxScaling = 1e4;
constexpr double kRhoMin = 1e-6, kRhoMax = 1e6, kRhoEq = 1e3, kRhoTol = 1e-4;
constexpr double kDivTol = 1e-30;

// Diagnostic build (-DMPCQ_STAMPS): thread 0 accumulates s_memtime deltas per
// phase into LaunchArgs::stamps.  The shipped build compiles these away.
#ifdef MPCQ_STAMPS
#define STAMP_DECL uint64_t st_acc[16] = {}; uint64_t st_last = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { if (threadIdx.x == 0) { const uint64_t nw_ = __builtin_amdgcn_s_memtime(); st_acc[i] += nw_ - st_last; st_last = nw_; } } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#endif

template <int N>
struct Geo {
  static constexpr int n = 24 * N, m = 44 * N, nnz = 126 * N - 18;
  static constexpr int NW = N / 4;  // waves per instance
  static constexpr int T = 64 * NW; // threads per instance
  static constexpr int RS = 3;      // row slots per lane  (176 rows / 64 lanes)
  static constexpr int CS = 2;      // column slots per lane (96 cols / 64 lanes)
};

// CSC offsets of MPC.create_ML's pattern (see oracle_pattern / mpcq_pattern).
template <int N>
__device__ __forceinline__ int XO(int k, int i) {  // state column X_{k+1}[i]
  return (k < N - 1) ? 30 * k + (i < 6 ? 2 * i : 12 + 3 * (i - 6)) : 30 * (N - 1) + i;
}
template <int N>
__device__ __forceinline__ int FO(int k, int f, int c) {  // force column f_k[3f+c]
  return 30 * N - 18 + 96 * k + 24 * f + 7 * c;
}
// stage-ordered index -> natural index of MPC.py's decision vector / rows
template <int N>
__device__ __forceinline__ int nat_col(int k, int j) {
  return j < 12 ? 12 * N + 12 * k + j : 12 * k + (j - 12);
}
template <int N>
__device__ __forceinline__ int nat_row(int k, int i) {
  return i < 12 ? 12 * k + i : (i < 24 ? 12 * N + 12 * k + (i - 12) : 24 * N + 20 * k + (i - 24));
}

// Visit the nonzeros of stage-ordered row (k, i): fn(csc position, stage-ordered column).
template <int N, class F>
__device__ __forceinline__ void for_row(int k, int i, F&& fn) {
  if (i < 12) {
    fn(XO<N>(k, i), 24 * k + 12 + i);
    if (k >= 1) {
      fn(XO<N>(k - 1, i) + (i < 6 ? 1 : 2), 24 * (k - 1) + 12 + i);
      if (i < 6) fn(XO<N>(k - 1, i + 6) + 1, 24 * (k - 1) + 18 + i);
    }
    if (i >= 6 && i < 9) {
      const int c = i - 6;
#pragma unroll
      for (int f = 0; f < 4; ++f) fn(FO<N>(k, f, c), 24 * k + 3 * f + c);
    } else if (i >= 9) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int c = 0; c < 3; ++c) fn(FO<N>(k, f, c) + i - 8, 24 * k + 3 * f + c);
    }
  } else if (i < 24) {
    const int q = i - 12;
    fn(FO<N>(k, q / 3, q % 3) + 4, 24 * k + q);
  } else {
    const int t = i - 24, f = t / 5, r = t % 5, cb = 24 * k + 3 * f;
    switch (r) {
      case 0: fn(FO<N>(k, f, 0) + 5, cb + 0); fn(FO<N>(k, f, 2) + 5, cb + 2); break;
      case 1: fn(FO<N>(k, f, 0) + 6, cb + 0); fn(FO<N>(k, f, 2) + 6, cb + 2); break;
      case 2: fn(FO<N>(k, f, 1) + 5, cb + 1); fn(FO<N>(k, f, 2) + 7, cb + 2); break;
      case 3: fn(FO<N>(k, f, 1) + 6, cb + 1); fn(FO<N>(k, f, 2) + 8, cb + 2); break;
      default: fn(FO<N>(k, f, 2) + 9, cb + 2); break;
    }
  }
}

// Visit the nonzeros of stage-local column (k, j): fn(csc position, stage-ordered row).
template <int N, class F>
__device__ __forceinline__ void for_col(int k, int j, F&& fn) {
  if (j >= 12) {
    const int i = j - 12, xo = XO<N>(k, i);
    fn(xo, 44 * k + i);
    if (k < N - 1) {
      if (i >= 6) {
        fn(xo + 1, 44 * (k + 1) + i - 6);
        fn(xo + 2, 44 * (k + 1) + i);
      } else {
        fn(xo + 1, 44 * (k + 1) + i);
      }
    }
  } else {
    const int f = j / 3, c = j % 3, fo = FO<N>(k, f, c), rb = 44 * k;
    fn(fo, rb + 6 + c);
    fn(fo + 1, rb + 9);
    fn(fo + 2, rb + 10);
    fn(fo + 3, rb + 11);
    fn(fo + 4, rb + 12 + j);
    const int fr = rb + 24 + 5 * f;
    if (c == 0) {
      fn(fo + 5, fr); fn(fo + 6, fr + 1);
    } else if (c == 1) {
      fn(fo + 5, fr + 2); fn(fo + 6, fr + 3);
    } else {
#pragma unroll
      for (int t = 0; t < 5; ++t) fn(fo + 5 + t, fr + t);
    }
  }
}

__device__ __forceinline__ void wave_sync() {
  // LDS is processed in order per wave; this only stops the compiler from
  // moving LDS accesses across the point and drains outstanding LDS ops.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

// ----------------------------------------------------------------------------
// Formulation pieces (restating MPC.py; see oracle/mpcq_oracle.c for the CPU twin)

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

// The 24 CSC values of foot f's three force columns in one stage
// (MPC.py:119-148 structure; B rows 9..11 = dt inv(Rz(yaw) gI) [lever]x,
// MPC.py:339-345; swing flag S (MPC.py:628)).
__device__ void form_foot(const mpcq_params& p, double yaw, double l0, double l1, double l2,
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

// Bounds of stage-ordered row (k, i) (MPC.py:197-232, 366-378, 410).
// xr = xref (12 x (N+1), row-major) staged in LDS.
template <int N>
__device__ void row_bounds(const mpcq_params& p, const double* xr, int k, int i, double& lo,
                           double& hi) {
  constexpr int NP1 = N + 1;
  if (i < 12) {
    const int r = i;
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
    v = v + dv;
    lo = v;
    hi = v;
  } else if (i < 24) {
    lo = 0.0;
    hi = 0.0;
  } else {
    hi = 0.0;
    lo = ((i - 24) % 5 == 4) ? -p.fz_max : -INFINITY;
  }
}

// ----------------------------------------------------------------------------
// Shared memory of one instance.

template <int N>
struct Smem {
  double Ab[Geo<N>::nnz];   // scaled constraint values, CSC order
  double Gam[N * 144];      // Gamma_k, 12x12 row-major
  double vn[Geo<N>::n];     // column-space exchange, stage ordered (24 per stage)
  double vm[Geo<N>::m];     // row-space exchange, stage ordered (44 per stage)
  double rh[Geo<N>::m];     // rho per row, stage ordered
  double sv[12 * N];        // forward recurrence (alpha -> s)
  double vv[12 * N];        // backward recurrence (beta -> v)
  double K0[576], K1[576];  // factorisation: K_k / Gauss-Jordan ping-pong (prologue: xref, fsteps)
  double Ch[288];           // C_k (24x12)
  double Tm[288];           // C_k Y_{k-1}
  double Y[144];            // Y_{k-1} = (S_{k-1}^{-1})_XX
  double Sc[256];           // per-stage structured copy of A for K_k
  double wsc[N / 4][64];    // per-wave scratch
  double red[N / 4][16];    // per-wave reduction partials
  int phase_of_stage[N];
  int contact[20][4];
  int flag[4];              // [0] formulation status, [1] factorisation failure
};

// Sc layout (per stage k, all scaled):
//   [0,72)    Bd[6][12]  dynamics rows 6..11 of stage k on its force columns
//   [72,84)   Xd[12]     dynamics row i of stage k on X_{k+1}[i]
//   [84,108)  Nd[12][2]  dynamics row i of stage k+1 on X_{k+1}[i] / X_{k+1}[i+6]
//   [108,120) Sw[12]     swing-mask rows
//   [120,180) Fr[4][5][3] friction rows (foot, row, component)
//   [180,192) rd  rho of dynamics rows of stage k
//   [192,204) rn  rho of dynamics rows of stage k+1
//   [204,216) rs  rho of swing rows
//   [216,236) rf  rho of friction rows
//   [236,248) Hd[12]     dynamics row i of stage k on X_k[i]      (from stage k-1's columns)
//   [248,254) Hd6[6]     dynamics row i of stage k on X_k[i+6]
enum { SC_BD = 0, SC_XD = 72, SC_ND = 84, SC_SW = 108, SC_FR = 120, SC_RD = 180, SC_RN = 192,
       SC_RS = 204, SC_RF = 216, SC_HD = 236, SC_HD6 = 248 };

// ----------------------------------------------------------------------------
// Factorisation of K = P + sigma I + A' diag(rh) A into the register-resident
// S_k^{-1} blocks and the LDS Gamma_k.  pd (P + sigma diagonal, stage ordered)
// must be in sh.vn.  Returns false on a non-positive pivot.

template <int N>
__device__ __forceinline__ bool factor(Smem<N>& sh, double (&Si)[4][12]) {
  constexpr int T = Geo<N>::T, NW = Geo<N>::NW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  bool ok = true;
  {
    for (int k = 0; k < N; ++k) {
      const int s = k / NW, w = k % NW;
      // --- 1. structured copy of the rows touching stage k
      for (int e = tid; e < 256; e += T) {
        double v = 0.0;
        if (e < SC_XD) {
          const int r = e / 12, a = e % 12, f = a / 3, c = a % 3;  // dyn row 6+r, force col a
          const int row = 6 + r;
          if (row < 9) v = (c == row - 6) ? sh.Ab[FO<N>(k, f, c)] : 0.0;
          else v = sh.Ab[FO<N>(k, f, c) + row - 8];
        } else if (e < SC_ND) {
          v = sh.Ab[XO<N>(k, e - SC_XD)];
        } else if (e < SC_SW) {
          const int q = e - SC_ND, i = q >> 1, h = q & 1;
          if (k < N - 1) {
            if (h == 0) v = sh.Ab[XO<N>(k, i) + (i < 6 ? 1 : 2)];
            else v = (i < 6) ? sh.Ab[XO<N>(k, i + 6) + 1] : 0.0;
          }
        } else if (e < SC_FR) {
          const int q = e - SC_SW;
          v = sh.Ab[FO<N>(k, q / 3, q % 3) + 4];
        } else if (e < SC_RD) {
          const int q = e - SC_FR, f = q / 15, t = (q % 15) / 3, c = q % 3;
          // friction row 5f+t on component c (C matrix, MPC.py:136-138)
          int off = -1;
          if (c == 0 && t < 2) off = 5 + t;
          else if (c == 1 && (t == 2 || t == 3)) off = 5 + (t - 2);
          else if (c == 2) off = 5 + t;
          v = off >= 0 ? sh.Ab[FO<N>(k, f, c) + off] : 0.0;
        } else if (e < SC_RN) {
          v = sh.rh[44 * k + (e - SC_RD)];
        } else if (e < SC_RS) {
          v = (k < N - 1) ? sh.rh[44 * (k + 1) + (e - SC_RN)] : 0.0;
        } else if (e < SC_RF) {
          v = sh.rh[44 * k + 12 + (e - SC_RS)];
        } else if (e < SC_HD) {
          v = sh.rh[44 * k + 24 + (e - SC_RF)];
        } else if (e < SC_HD6) {
          const int i = e - SC_HD;
          v = (k >= 1) ? sh.Ab[XO<N>(k - 1, i) + (i < 6 ? 1 : 2)] : 0.0;
        } else if (e < SC_HD6 + 6) {
          const int i = e - SC_HD6;
          v = (k >= 1) ? sh.Ab[XO<N>(k - 1, i + 6) + 1] : 0.0;
        }
        sh.Sc[e] = v;
      }
      __syncthreads();
      const double* Sc = sh.Sc;
      // --- 2. K_k (without the Schur term) and C_k
      for (int e = tid; e < 576 + 288; e += T) {
        if (e < 576) {
          const int a = e / 24, b = e % 24;
          double v = 0.0;
          if (a < 12 && b < 12) {
#pragma unroll
            for (int r = 0; r < 6; ++r)
              v += Sc[SC_RD + 6 + r] * Sc[SC_BD + 12 * r + a] * Sc[SC_BD + 12 * r + b];
            if (a == b) v += Sc[SC_RS + a] * Sc[SC_SW + a] * Sc[SC_SW + a] + sh.vn[24 * k + a];
            const int fa = a / 3, fb = b / 3, ca = a % 3, cb = b % 3;
            if (fa == fb) {
#pragma unroll
              for (int t = 0; t < 5; ++t)
                v += Sc[SC_RF + 5 * fa + t] * Sc[SC_FR + 15 * fa + 3 * t + ca] *
                     Sc[SC_FR + 15 * fa + 3 * t + cb];
            }
          } else if (a < 12 || b < 12) {
            const int fa = a < 12 ? a : b, i = (a < 12 ? b : a) - 12;
            if (i >= 6) v = Sc[SC_RD + i] * Sc[SC_BD + 12 * (i - 6) + fa] * Sc[SC_XD + i];
          } else {
            const int i = a - 12, i2 = b - 12;
            if (i == i2) v = Sc[SC_RD + i] * Sc[SC_XD + i] * Sc[SC_XD + i] + sh.vn[24 * k + a];
            // dynamics rows of stage k+1: row r' touches X[r'] (Nd[r'][0]) and X[r'+6] (Nd[r'][1])
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int rp = h == 0 ? i : i - 6;
              if (rp >= 0) {
                const double c1 = (i == rp) ? Sc[SC_ND + 2 * rp] : (rp < 6 ? Sc[SC_ND + 2 * rp + 1] : 0.0);
                double c2 = 0.0;
                if (i2 == rp) c2 = Sc[SC_ND + 2 * rp];
                else if (i2 == rp + 6 && rp < 6) c2 = Sc[SC_ND + 2 * rp + 1];
                v += Sc[SC_RN + rp] * c1 * c2;
              }
            }
          }
          sh.K0[e] = v;
        } else if (k >= 1) {
          // C_k[j][i'] = sum_i E(i, j) rho_i H(i, i'),  i in {i', i'-6}
          const int q = e - 576, j = q / 12, ip = q % 12;
          double v = 0.0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = h == 0 ? ip : ip - 6;
            if (i < 0) continue;
            const double H = (h == 0) ? Sc[SC_HD + ip] : Sc[SC_HD6 + i];
            double E = 0.0;
            if (j < 12) {
              if (i >= 6) E = Sc[SC_BD + 12 * (i - 6) + j];
            } else if (j - 12 == i) {
              E = Sc[SC_XD + i];
            }
            v += E * Sc[SC_RD + i] * H;
          }
          sh.Ch[q] = v;
        }
      }
      __syncthreads();
      if (k >= 1) {
        for (int e = tid; e < 288; e += T) {  // Tm = C_k Y_{k-1}
          const int a = e / 12, ip = e % 12;
          double v = 0.0;
#pragma unroll
          for (int t = 0; t < 12; ++t) v += sh.Ch[12 * a + t] * sh.Y[12 * t + ip];
          sh.Tm[e] = v;
        }
        __syncthreads();
        for (int e = tid; e < 576; e += T) {  // K -= Tm C_k'
          const int a = e / 24, b = e % 24;
          double v = 0.0;
#pragma unroll
          for (int t = 0; t < 12; ++t) v += sh.Tm[12 * a + t] * sh.Ch[12 * b + t];
          sh.K0[e] -= v;
        }
        __syncthreads();
      }
      // --- 3. in-place Gauss-Jordan inverse (SPD, no pivoting), ping-pong K0 <-> K1
      for (int p = 0; p < 24; ++p) {
        const double* src = (p & 1) ? sh.K1 : sh.K0;
        double* dst = (p & 1) ? sh.K0 : sh.K1;
        const double d = src[25 * p];
        if (!(d > 0.0)) ok = false;
        const double id = 1.0 / d;
        for (int e = tid; e < 576; e += T) {
          const int a = e / 24, b = e % 24;
          double v;
          if (a == p && b == p) v = id;
          else if (a == p) v = src[e] * id;
          else if (b == p) v = -src[e] * id;
          else v = src[e] - src[24 * a + p] * src[24 * p + b] * id;
          dst[e] = v;
        }
        __syncthreads();
      }
      // S_k^{-1} now in K0 (24 passes).  Y_k, Gamma_k, owner registers.
      for (int e = tid; e < 288; e += T) {
        if (e < 144) {
          const int i = e / 12, ip = e % 12;
          sh.Y[e] = sh.K0[24 * (12 + i) + 12 + ip];
        } else {
          const int q = e - 144, i = q / 12, ip = q % 12;
          double v = 0.0;
          if (k >= 1) {
#pragma unroll
            for (int t = 0; t < 24; ++t) v += sh.K0[24 * (12 + i) + t] * sh.Ch[12 * t + ip];
          }
          sh.Gam[144 * k + q] = v;
        }
      }
      if (wv == w && lane < 48) {  // switch keeps the register index compile-time
        const double* src = sh.K0 + 24 * (lane >> 1) + 12 * (lane & 1);
        switch (s) {
#define MPCQ_LOAD_SLOT(S_)                                   \
  case S_:                                                   \
    _Pragma("unroll") for (int c = 0; c < 12; ++c) Si[S_][c] = src[c]; \
    break;
          MPCQ_LOAD_SLOT(0)
          MPCQ_LOAD_SLOT(1)
          MPCQ_LOAD_SLOT(2)
          MPCQ_LOAD_SLOT(3)
#undef MPCQ_LOAD_SLOT
        }
      }
      __syncthreads();
    }
  }
  return ok;
}

// ----------------------------------------------------------------------------
// KKT solve: b in sh.vn (stage ordered) -> w in sh.vn.

#ifdef MPCQ_STAMPS
#define KKT_STAMP_ARGS , uint64_t (&st_acc)[16], uint64_t& st_last
#define KKT_STAMP_PASS , st_acc, st_last
#else
#define KKT_STAMP_ARGS
#define KKT_STAMP_PASS
#endif
template <int N>
__device__ __forceinline__ void kkt_solve(Smem<N>& sh, const double (&Si)[4][12] KKT_STAMP_ARGS) {
  constexpr int NW = Geo<N>::NW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane >> 1, h = lane & 1;
  double* ws = sh.wsc[wv];
  // phase A: alpha_k = (S_k^{-1})_{X,:} b_k
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = s * NW + wv;
    double acc = 0.0;
    if (lane >= 24 && lane < 48) {
#pragma unroll
      for (int c = 0; c < 12; ++c) acc += Si[s][c] * sh.vn[24 * k + 12 * h + c];
    }
    acc += __shfl_xor(acc, 1);
    if (lane >= 24 && lane < 48 && h == 0) sh.sv[12 * k + r - 12] = acc;
  }
  __syncthreads();
  STAMP(4);
  // forward recurrence s_k = alpha_k - Gamma_k s_{k-1} (wave 0)
  if (wv == 0) {
    const int i = lane >> 2, q = lane & 3;
    const bool act = lane < 48;
    double p0 = 0.0, p1 = 0.0, p2 = 0.0;
    for (int k = 0; k < N; ++k) {
      double a = 0.0, acc = 0.0;
      if (act) {
        a = sh.sv[12 * k + i];
        const double* G = sh.Gam + 144 * k + 12 * i + 3 * q;
        acc = G[0] * p0 + G[1] * p1 + G[2] * p2;
      }
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      const double si = a - acc;
      if (act && q == 0) sh.sv[12 * k + i] = si;
      p0 = __shfl(si, 4 * (3 * q + 0));
      p1 = __shfl(si, 4 * (3 * q + 1));
      p2 = __shfl(si, 4 * (3 * q + 2));
    }
  }
  __syncthreads();
  STAMP(5);
  // phase B: t_k = S_k^{-1}(b_k - C_k s_{k-1}); beta_k = C_k' t_k
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = s * NW + wv;
    if (k >= 1 && lane < 12) {  // u = rho_dyn (H s_{k-1})
      const int i = lane;
      double v = sh.Ab[XO<N>(k - 1, i) + (i < 6 ? 1 : 2)] * sh.sv[12 * (k - 1) + i];
      if (i < 6) v += sh.Ab[XO<N>(k - 1, i + 6) + 1] * sh.sv[12 * (k - 1) + i + 6];
      ws[i] = sh.rh[44 * k + i] * v;
    }
    wave_sync();
    if (lane < 24) {  // bhat = b - C_k s_{k-1}
      const int j = lane;
      double cs = 0.0;
      if (k >= 1) {
        if (j < 12) {
          const int f = j / 3, c = j % 3, fo = FO<N>(k, f, c);
          cs = sh.Ab[fo] * ws[6 + c] + sh.Ab[fo + 1] * ws[9] + sh.Ab[fo + 2] * ws[10] +
               sh.Ab[fo + 3] * ws[11];
        } else {
          cs = sh.Ab[XO<N>(k, j - 12)] * ws[j - 12];
        }
      }
      ws[16 + j] = sh.vn[24 * k + j] - cs;
    }
    wave_sync();
    double acc = 0.0;
    if (lane < 48) {
#pragma unroll
      for (int c = 0; c < 12; ++c) acc += Si[s][c] * ws[16 + 12 * h + c];
    }
    acc += __shfl_xor(acc, 1);
    if (lane < 48 && h == 0) sh.vn[24 * k + r] = acc;
    wave_sync();
    if (k >= 1) {
      if (lane < 12) {  // u_i = rho_i (dynamics row k, i) . t_k
        const int i = lane;
        const double* t = sh.vn + 24 * k;
        double v = sh.Ab[XO<N>(k, i)] * t[12 + i];
        if (i >= 6 && i < 9) {
          const int c = i - 6;
#pragma unroll
          for (int f = 0; f < 4; ++f) v += sh.Ab[FO<N>(k, f, c)] * t[3 * f + c];
        } else if (i >= 9) {
#pragma unroll
          for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int c = 0; c < 3; ++c) v += sh.Ab[FO<N>(k, f, c) + i - 8] * t[3 * f + c];
        }
        ws[48 + i] = sh.rh[44 * k + i] * v;
      }
      wave_sync();
      if (lane < 12) {  // beta_k[i'] = sum_i H(i, i') u_i
        const int ip = lane;
        double v = sh.Ab[XO<N>(k - 1, ip) + (ip < 6 ? 1 : 2)] * ws[48 + ip];
        if (ip >= 6) v += sh.Ab[XO<N>(k - 1, ip) + 1] * ws[48 + ip - 6];
        sh.vv[12 * (k - 1) + ip] = v;
      }
    }
    wave_sync();
  }
  __syncthreads();
  STAMP(6);
  // backward recurrence v_{k-1} = beta_k - Gamma_k' v_k (wave 0)
  if (wv == 0) {
    const int i = lane >> 2, q = lane & 3;
    const bool act = lane < 48;
    double p0 = 0.0, p1 = 0.0, p2 = 0.0;
    for (int k = N - 1; k >= 1; --k) {
      double bt = 0.0, acc = 0.0;
      if (act) {
        bt = sh.vv[12 * (k - 1) + i];
        const double* G = sh.Gam + 144 * k + i;
        acc = G[12 * (3 * q + 0)] * p0 + G[12 * (3 * q + 1)] * p1 + G[12 * (3 * q + 2)] * p2;
      }
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      const double vi = bt - acc;
      if (act && q == 0) sh.vv[12 * (k - 1) + i] = vi;
      p0 = __shfl(vi, 4 * (3 * q + 0));
      p1 = __shfl(vi, 4 * (3 * q + 1));
      p2 = __shfl(vi, 4 * (3 * q + 2));
    }
  }
  __syncthreads();
  STAMP(7);
  // phase C: w_k = t_k - (S_k^{-1})_{:,X} v_k
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = s * NW + wv;
    if (k < N - 1 && lane < 48 && h == 1) {
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < 12; ++c) acc += Si[s][c] * sh.vv[12 * k + c];
      sh.vn[24 * k + r] -= acc;
    }
  }
  __syncthreads();
  STAMP(8);
}

// ----------------------------------------------------------------------------
// The engine kernel: one workgroup per instance.
//   FUSED  = true : formulate from (xref, fsteps) then solve   (MPC.run)
//   FUSED  = false: solve the given (Ax, l, u)                  (osqp update+solve)
//   SOLVE  = false: formulation only, write Ax / l / u          (update_matrices)

template <int N, bool FUSED, bool SOLVE>
__global__ __launch_bounds__(16 * N, 2) void engine_kernel(mpcq_params p, LaunchArgs a) {
  constexpr int n = Geo<N>::n, m = Geo<N>::m, nnz = Geo<N>::nnz;
  constexpr int T = Geo<N>::T, NW = Geo<N>::NW, RS = Geo<N>::RS, CS = Geo<N>::CS;
  __shared__ Smem<N> sh;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t b = blockIdx.x;
  if (b >= a.batch) return;
  STAMP_DECL

  // slot bookkeeping (rows / columns of this wave's stages)
  int rK[RS], rI[RS], cK[CS], cJ[CS];
  bool rV[RS], cV[CS];
#pragma unroll
  for (int t = 0; t < RS; ++t) {
    const int q = lane + 64 * t;
    rV[t] = q < 176;
    rK[t] = (q / 44) * NW + wv;
    rI[t] = q % 44;
    if (!rV[t]) { rK[t] = 0; rI[t] = 0; }
  }
#pragma unroll
  for (int t = 0; t < CS; ++t) {
    const int q = lane + 64 * t;
    cV[t] = q < 96;
    cK[t] = (q / 24) * NW + wv;
    cJ[t] = q % 24;
    if (!cV[t]) { cK[t] = 0; cJ[t] = 0; }
  }
  double lo[RS], hi[RS];

  if (tid == 0) { sh.flag[0] = 0; sh.flag[1] = 0; }

  // ---------------------------------------------------------------- prologue
  if (FUSED || !SOLVE) {
    // stage xref / fsteps in LDS (K0 / K1 are free until the first factorisation)
    double* xr = sh.K0;
    double* fs = sh.K1;
    const double* gx = a.xref + b * 12 * (N + 1);
    const double* gf = a.fsteps + b * 260;
    for (int e = tid; e < 12 * (N + 1); e += T) xr[e] = gx[e];
    for (int e = tid; e < 260; e += T) fs[e] = gf[e];
    __syncthreads();
    if (tid == 0) {  // construct_gait + phase walk (MPC.py:635-652, 336-352, 626-631)
      int idx = -1;
      for (int j = 0; j < 20; ++j)
        if (fs[13 * j] == 0.0) { idx = j; break; }
      int bad = idx < 0;
      int k = 0;
      for (int j = 0; j < (idx < 0 ? 0 : idx) && !bad; ++j) {
        const double d = fs[13 * j];
        if (!(fabs(d) < 1e6)) { bad = 1; break; }
        const int di = (int)d;
        if (di < 0) { bad = 1; break; }
        for (int f = 0; f < 4; ++f) {
          const double x = fs[13 * j + 1 + 3 * f];
          sh.contact[j][f] = !(isnan(x) || x == 0.0);
        }
        for (int t = 0; t < di; ++t, ++k)
          if (k < N) sh.phase_of_stage[k] = j;
      }
      if (k != N) bad = 1;
      sh.flag[0] = bad ? MPCQ_STATUS_BAD_GAIT : 0;
    }
    __syncthreads();
    const bool bad = sh.flag[0] != 0;
    if (!bad) {
      for (int c = tid; c < 12 * N; c += T) {  // state columns: -I / A (MPC.py:107-115)
        const int k = c / 12, i = c % 12, xo = XO<N>(k, i);
        sh.Ab[xo] = -1.0;
        if (k < N - 1) {
          if (i >= 6) { sh.Ab[xo + 1] = p.dt; sh.Ab[xo + 2] = 1.0; }
          else sh.Ab[xo + 1] = 1.0;
        }
      }
      for (int e = tid; e < 4 * N; e += T) {  // force columns, one foot per thread
        const int k = e >> 2, f = e & 3, j = sh.phase_of_stage[k];
        double lv[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          double ft;
          if (a.mode == MPCQ_MODE_SETUP) ft = p.footholds[4 * r + f];
          else {
            ft = fs[13 * j + 1 + 3 * f + r];
            if (isnan(ft)) ft = 0.0;  // MPC.py:327
          }
          lv[r] = ft - xr[r * (N + 1) + k];
        }
        form_foot(p, xr[5 * (N + 1) + k], lv[0], lv[1], lv[2], 1.0 - (double)sh.contact[j][f],
                  sh.Ab + FO<N>(k, f, 0));
      }
#pragma unroll
      for (int t = 0; t < RS; ++t)
        if (rV[t]) row_bounds<N>(p, xr, rK[t], rI[t], lo[t], hi[t]);
    }
    if (!SOLVE) {
      __syncthreads();
      if (tid == 0 && a.status) a.status[b] = sh.flag[0];
      if (bad) return;
      double* go = a.Ax_out + b * nnz;
      for (int e = tid; e < nnz; e += T) go[e] = sh.Ab[e];
#pragma unroll
      for (int t = 0; t < RS; ++t)
        if (rV[t]) {
          const int R = nat_row<N>(rK[t], rI[t]);
          a.l_out[b * m + R] = lo[t];
          a.u_out[b * m + R] = hi[t];
        }
      return;
    }
  } else {
    const double* ga = a.Ax + b * nnz;
    for (int e = tid; e < nnz; e += T) sh.Ab[e] = ga[e];
#pragma unroll
    for (int t = 0; t < RS; ++t) {
      lo[t] = 0.0; hi[t] = 0.0;
      if (rV[t]) {
        const int R = nat_row<N>(rK[t], rI[t]);
        lo[t] = a.l[b * m + R];
        hi[t] = a.u[b * m + R];
      }
    }
  }
  if constexpr (SOLVE) {
    __syncthreads();
    int status = sh.flag[0];
    // ------------------------------------------------------------ checks
    {
      int bad = 0;
      for (int e = tid; e < nnz; e += T)
        if (!isfinite(sh.Ab[e])) bad = 1;
#pragma unroll
      for (int t = 0; t < RS; ++t) {
        if (!rV[t]) continue;
        if (isnan(lo[t]) || isnan(hi[t])) bad = 1;
        lo[t] = lo[t] < -kInf ? -kInf : lo[t];
        hi[t] = hi[t] > kInf ? kInf : hi[t];
      }
      if (bad) atomicOr(&sh.flag[1], 1);
      __syncthreads();
      if (status == 0 && sh.flag[1]) status = MPCQ_STATUS_NONFINITE;
      __syncthreads();
      if (tid == 0) sh.flag[1] = 0;
    }
    double x[CS], D[CS], Pb[CS];
    double z[RS], y[RS], E[RS], rho[RS], rinv[RS];
    int ct[RS];
#pragma unroll
    for (int t = 0; t < CS; ++t) {
      x[t] = 0.0; D[t] = 1.0;
      Pb[t] = cJ[t] < 12 ? p.force_weight : p.state_weights[cJ[t] - 12];
    }
#pragma unroll
    for (int t = 0; t < RS; ++t) { z[t] = 0.0; y[t] = 0.0; E[t] = 1.0; rho[t] = 0.0; rinv[t] = 0.0; ct[t] = 0; }
    double cscale = 1.0;
    double Si[4][12];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < 12; ++c) Si[s][c] = 0.0;
    int it_done = 0, n_upd = 0;
    double rho_s = a.rho_in ? a.rho_in[b] : p.rho;
    rho_s = fmin(fmax(rho_s, kRhoMin), kRhoMax);

    if (status == 0) {
      __syncthreads();
      STAMP(0);
      // ---------------------------------------------------------- Ruiz scaling
      for (int it = 0; it < p.scaling; ++it) {
        double psum = 0.0;
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          if (!cV[t]) continue;
          double v = fabs(Pb[t]);
          for_col<N>(cK[t], cJ[t], [&](int pos, int) { v = fmax(v, fabs(sh.Ab[pos])); });
          v = v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v);
          const double dt = 1.0 / sqrt(v);
          sh.vn[24 * cK[t] + cJ[t]] = dt;
          D[t] *= dt;
          Pb[t] = dt * Pb[t] * dt;
        }
#pragma unroll
        for (int t = 0; t < RS; ++t) {
          if (!rV[t]) continue;
          double v = 0.0;
          for_row<N>(rK[t], rI[t], [&](int pos, int) { v = fmax(v, fabs(sh.Ab[pos])); });
          v = v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v);
          const double et = 1.0 / sqrt(v);
          sh.vm[44 * rK[t] + rI[t]] = et;
          E[t] *= et;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          if (!cV[t]) continue;
          const double dt = sh.vn[24 * cK[t] + cJ[t]];
          for_col<N>(cK[t], cJ[t], [&](int pos, int R) { sh.Ab[pos] = sh.vm[R] * sh.Ab[pos] * dt; });
          psum += fabs(Pb[t]);
        }
        psum = wave_sum(psum);
        if (lane == 0) sh.red[wv][0] = psum;
        __syncthreads();
        double tot = 0.0;
#pragma unroll
        for (int w = 0; w < NW; ++w) tot += sh.red[w][0];
        const double mean = tot / n;
        double ctmp = mean > 1.0 ? mean : 1.0;
        ctmp = ctmp < kMinScaling ? 1.0 : (ctmp > kMaxScaling ? kMaxScaling : ctmp);
        ctmp = 1.0 / ctmp;
#pragma unroll
        for (int t = 0; t < CS; ++t) Pb[t] *= ctmp;
        cscale *= ctmp;
        __syncthreads();
      }
      // scaled bounds, constraint types, rho per row (osqp set_rho_vec)
#pragma unroll
      for (int t = 0; t < RS; ++t) {
        if (!rV[t]) continue;
        lo[t] *= E[t];
        hi[t] *= E[t];
        if (lo[t] < -kInf * kMinScaling && hi[t] > kInf * kMinScaling) ct[t] = -1;
        else if (hi[t] - lo[t] < kRhoTol) ct[t] = 1;
        else ct[t] = 0;
        rho[t] = ct[t] == -1 ? kRhoMin : (ct[t] == 1 ? kRhoEq * rho_s : rho_s);
        rinv[t] = 1.0 / rho[t];
        sh.rh[44 * rK[t] + rI[t]] = rho[t];
      }
      // warm start (osqp_warm_start: x = D^-1 x0, z = A x; y = c E^-1 y0)
      if (a.warm_x) {
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          if (!cV[t]) continue;
          x[t] = a.warm_x[b * n + nat_col<N>(cK[t], cJ[t])] / D[t];
          sh.vn[24 * cK[t] + cJ[t]] = x[t];
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < RS; ++t) {
          if (!rV[t]) continue;
          double v = 0.0;
          for_row<N>(rK[t], rI[t], [&](int pos, int C) { v += sh.Ab[pos] * sh.vn[C]; });
          z[t] = v;
        }
        __syncthreads();
      }
      if (a.warm_y) {
#pragma unroll
        for (int t = 0; t < RS; ++t)
          if (rV[t]) y[t] = cscale * a.warm_y[b * m + nat_row<N>(rK[t], rI[t])] / E[t];
      }
      // ---------------------------------------------------------- factorise
#pragma unroll
      for (int t = 0; t < CS; ++t)
        if (cV[t]) sh.vn[24 * cK[t] + cJ[t]] = Pb[t] + p.sigma;
      __syncthreads();
      STAMP(1);
      if (!factor<N>(sh, Si)) status = MPCQ_STATUS_FACTOR_FAILED;
      STAMP(2);

      // ---------------------------------------------------------- ADMM
      double pri_res = 0.0, dua_res = 0.0, eps_pri = 0.0, eps_dua = 0.0;
      double s_pri = 0.0, s_dua = 0.0;
      bool can_check = false;
      auto update_info = [&]() {
        // x -> vn, y -> vm
#pragma unroll
        for (int t = 0; t < CS; ++t)
          if (cV[t]) sh.vn[24 * cK[t] + cJ[t]] = x[t];
#pragma unroll
        for (int t = 0; t < RS; ++t)
          if (rV[t]) sh.vm[44 * rK[t] + rI[t]] = y[t];
        __syncthreads();
        double q[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) q[e] = 0.0;
#pragma unroll
        for (int t = 0; t < RS; ++t) {
          if (!rV[t]) continue;
          double ax = 0.0;
          for_row<N>(rK[t], rI[t], [&](int pos, int C) { ax += sh.Ab[pos] * sh.vn[C]; });
          const double ei = 1.0 / E[t], d = ax - z[t];
          q[0] = fmax(q[0], fabs(ei * d));
          q[1] = fmax(q[1], fabs(ei * ax));
          q[2] = fmax(q[2], fabs(ei * z[t]));
          q[3] = fmax(q[3], fabs(d));
          q[4] = fmax(q[4], fabs(ax));
          q[5] = fmax(q[5], fabs(z[t]));
        }
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          if (!cV[t]) continue;
          double aty = 0.0;
          for_col<N>(cK[t], cJ[t], [&](int pos, int R) { aty += sh.Ab[pos] * sh.vm[R]; });
          const double px = Pb[t] * x[t], di = 1.0 / D[t], d = px + 0.0 + aty;
          q[6] = fmax(q[6], fabs(di * d));
          q[7] = fmax(q[7], fabs(di * px));
          q[8] = fmax(q[8], fabs(di * aty));
          q[9] = fmax(q[9], fabs(d));
          q[10] = fmax(q[10], fabs(px));
          q[11] = fmax(q[11], fabs(aty));
        }
#pragma unroll
        for (int e = 0; e < 12; ++e) {
          const double v = wave_max(q[e]);
          if (lane == 0) sh.red[wv][e] = v;
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 12; ++e) {
          double v = 0.0;
#pragma unroll
          for (int w = 0; w < NW; ++w) v = fmax(v, sh.red[w][e]);
          q[e] = v;
        }
        const double cinv = 1.0 / cscale;
        pri_res = q[0];
        dua_res = cinv * q[6];
        eps_pri = p.eps_abs + p.eps_rel * fmax(q[1], q[2]);
        eps_dua = p.eps_abs + p.eps_rel * cinv * fmax(q[7], q[8]);
        s_pri = q[3] / (fmax(q[4], q[5]) + kDivTol);
        s_dua = q[9] / (fmax(q[10], q[11]) + kDivTol);
        __syncthreads();
      };
      auto converged = [&](double f) { return pri_res < f * eps_pri && dua_res < f * eps_dua; };

      int iter = 1;
      for (; status == 0 && iter <= p.max_iter; ++iter) {
        // w = rho z - y (z, y from the previous iterate)
#pragma unroll
        for (int t = 0; t < RS; ++t)
          if (rV[t]) sh.vm[44 * rK[t] + rI[t]] = rho[t] * z[t] - y[t];
        __syncthreads();
        STAMP(3);
        // b = sigma x - q + A' w
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          if (!cV[t]) continue;
          double v = 0.0;
          for_col<N>(cK[t], cJ[t], [&](int pos, int R) { v += sh.Ab[pos] * sh.vm[R]; });
          sh.vn[24 * cK[t] + cJ[t]] = p.sigma * x[t] + v;
        }
        wave_sync();
        kkt_solve<N>(sh, Si KKT_STAMP_PASS);
        // z update, y update (osqp update_z / update_y); x update
#pragma unroll
        for (int t = 0; t < RS; ++t) {
          if (!rV[t]) continue;
          double zt = 0.0;
          for_row<N>(rK[t], rI[t], [&](int pos, int C) { zt += sh.Ab[pos] * sh.vn[C]; });
          const double zr = p.alpha * zt + (1.0 - p.alpha) * z[t];
          const double tt = zr + y[t] * rinv[t];
          const double zn = tt < lo[t] ? lo[t] : (tt > hi[t] ? hi[t] : tt);
          y[t] = y[t] + rho[t] * (zr - zn);
          z[t] = zn;
        }
#pragma unroll
        for (int t = 0; t < CS; ++t)
          if (cV[t]) x[t] = p.alpha * sh.vn[24 * cK[t] + cJ[t]] + (1.0 - p.alpha) * x[t];
        can_check = p.check_termination > 0 && (iter % p.check_termination == 0);
        const bool adapt = p.adaptive_rho && p.adaptive_rho_interval > 0 &&
                           (iter % p.adaptive_rho_interval == 0);
        STAMP(9);
        if (can_check || adapt) {
          __syncthreads();  // vn (w) fully consumed before update_info reuses it
          update_info();
          if (!(isfinite(pri_res) && isfinite(dua_res))) { status = MPCQ_STATUS_NONFINITE; break; }
          if (can_check && converged(1.0)) { status = MPCQ_STATUS_SOLVED; break; }
          if (adapt) {
            double rn = rho_s * sqrt(s_pri / (s_dua + kDivTol));
            rn = fmin(fmax(rn, kRhoMin), kRhoMax);
            if (rn > rho_s * p.adaptive_rho_tolerance || rn < rho_s / p.adaptive_rho_tolerance) {
              rho_s = rn;
#pragma unroll
              for (int t = 0; t < RS; ++t) {
                if (!rV[t]) continue;
                rho[t] = ct[t] == -1 ? kRhoMin : (ct[t] == 1 ? kRhoEq * rho_s : rho_s);
                rinv[t] = 1.0 / rho[t];
                sh.rh[44 * rK[t] + rI[t]] = rho[t];
              }
#pragma unroll
              for (int t = 0; t < CS; ++t)
                if (cV[t]) sh.vn[24 * cK[t] + cJ[t]] = Pb[t] + p.sigma;
              __syncthreads();
              STAMP(10);
              if (!factor<N>(sh, Si)) { status = MPCQ_STATUS_FACTOR_FAILED; break; }
              STAMP(2);
              ++n_upd;
            }
          }
        }
        __syncthreads();
        STAMP(10);
      }
      it_done = iter > p.max_iter ? p.max_iter : iter;
      if (status == 0) {
        __syncthreads();
        if (!can_check) {
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
    for (int t = 0; t < CS; ++t) {
      if (!cV[t]) continue;
      const double xv = nan_out ? NAN : D[t] * x[t];
      const int C = nat_col<N>(cK[t], cJ[t]);
      if (a.x) a.x[b * n + C] = xv;
      if (a.f0 && cK[t] == 0 && cJ[t] < 12) a.f0[b * 12 + cJ[t]] = xv;
    }
    if (a.y) {
#pragma unroll
      for (int t = 0; t < RS; ++t)
        if (rV[t]) a.y[b * m + nat_row<N>(rK[t], rI[t])] = nan_out ? NAN : E[t] * y[t] / cscale;
    }
#ifdef MPCQ_STAMPS
    STAMP(11);
    if (tid == 0 && a.stamps) {
      for (int i = 0; i < 16; ++i) a.stamps[b * 16 + i] = st_acc[i];
    }
#endif
    if (tid == 0) {
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
  const dim3 grid((unsigned)a.batch), block(Geo<N>::T);
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
