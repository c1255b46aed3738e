// mpcq_engine.hip — batched convex-MPC QP engine for MI355X (gfx950, CDNA4).
//
// One workgroup of N/4 wave64s owns one QP instance for its whole life:
// formulation (MPC.py:98-378), Ruiz scaling, KKT factorisation and the
// OSQP-0.6 ADMM iterations run out of registers + LDS.  HBM sees only the
// compulsory inputs (xref, fsteps) and outputs (f0 / x / y / status).
//
// Lane layout: a stage k is one 16-lane DPP row (so a wave holds 4 stages);
// lane s = 4f + c of row k is foot f, component c.  Lanes c < 3 own the
// column pair (force f_k[3f+c], state X_{k+1}[3f+c]) and three rows: the
// dynamics row 3f+c, the swing row 3f+c and friction row c of foot f; lane
// c = 3 owns friction rows 3 and 4 of foot f (its column work is a discarded
// shadow of lane c = 2).  Stage-wide vectors move by DPP row_newbcast,
// foot-wide ones by quad_perm; only stage-to-stage hand-offs go through LDS.
//
// KKT solve (P + sigma I + A' R A) w = b.  In stage order the matrix is block
// tridiagonal; the forces only couple inside a stage, so they are eliminated
// first (every stage in parallel: F_k = K_ff,k^{-1}, one row per lane), which
// leaves a block-tridiagonal system in the states with 12x12 blocks
//   D_k = K_XX,k - Xd Q_k Xd - Hd_{k+1} Q_{k+1} Hd_{k+1},   Q_k = W_k' F_k W_k (6x6)
//   L_k = C_X,k  - Xd Q_k Hd_k                              (W_k = R B_k on rows 6..11)
// factored two-ended ("twisted"): top-down for stages < m, bottom-up for
// stages > m, meeting at m = N/2, so each substitution sweep is N/2 steps deep:
//   y_k = b_k - G_k y_{k-1}   (k < m)      v_k = b_k - H_k v_{k+1}   (k > m)
//   x_m = M^{-1}(y_m + v_m - b_m)
//   x_k = S_k^{-1} y_k - G_{k+1}' x_{k+1}  x_k = U_k^{-1} v_k - H_{k-1}' x_{k-1}
// The two sweeps run at once in rows 0 and 1 of wave 0 (one instruction
// stream), reading G / H from LDS; S^{-1}, U^{-1}, M^{-1} rows stay in the
// stage lanes' registers.
#include <math.h>

#include <type_traits>
#include <utility>

#include "mpcq_internal.h"

namespace mpcq {
namespace {

// LDS views used by the loops.  Reads of loop-invariant data (the scaled A,
// the sweep matrices) go through these pointers, which the loops launder with
// an empty asm so the compiler re-reads LDS instead of hoisting dozens of
// invariant values into registers.
typedef __attribute__((address_space(3))) const double lds_cd;
typedef __attribute__((address_space(3))) double lds_d;
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const dbl2 lds_cd2;
// the per-instance workspace (N > 32) in the global address space: generic (flat)
// loads would also count in lgkmcnt, so every LDS wait behind them would wait for L2
typedef __attribute__((address_space(1))) const double g_cd;
typedef __attribute__((address_space(1))) double g_d;
typedef __attribute__((address_space(1))) const dbl2 g_cd2;

constexpr double kInf = 1e30;  // OSQP_INFTY
constexpr double kMinScaling = 1e-4, kMaxScaling = 1e4;
constexpr double kRhoMin = 1e-6, kRhoMax = 1e6, kRhoEq = 1e3, kRhoTol = 1e-4;
constexpr double kDivTol = 1e-30;

// constraint classes (OSQP set_rho_vec)
enum : unsigned { RC_LOOSE = 0, RC_INEQ = 1, RC_EQ = 2 };

#if defined(MPCQ_STAMPS) && defined(MPCQ_STAMPS_LEAN)
// lean variant: only the uniform points after the loop's barriers (1 prologue, 2 factor,
// 3 P1-P4, 7 sweeps, 10 P8-P9, 11 checks, 12 epilogue), accumulated in SGPRs without a
// lane branch, so the measured code stays close to the production build
#define STAMP_DECL uint64_t st_acc[16] = {}; uint64_t st_last = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { if constexpr ((i) == 1 || (i) == 2 || (i) == 3 || (i) == 7 || (i) == 10 || (i) == 11 || (i) == 12) { \
    const uint64_t nw_ = __builtin_amdgcn_s_memtime(); st_acc[i] += nw_ - st_last; st_last = nw_; } } while (0)
#elif defined(MPCQ_STAMPS)
// (MPCQ_STAMP_WAVE = w: the stamps of wave w's first lane instead of wave 0's, clamped
// to the workgroup's last wave: kStampT)
#define STAMP_DECL uint64_t st_acc[16] = {}; uint64_t st_last = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { if (threadIdx.x == kStampT) { const uint64_t nw_ = __builtin_amdgcn_s_memtime(); st_acc[i] += nw_ - st_last; st_last = nw_; } } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// CSC offsets of MPC.create_ML's pattern (see mpcq_pattern in mpcq_api.cpp).
template <int N>
__device__ __forceinline__ int XO(int k, int i) {  // state column X_{k+1}[i]
  return (k < N - 1) ? 30 * k + (i < 6 ? 2 * i : 12 + 3 * (i - 6)) : 30 * (N - 1) + i;
}
template <int N>
__device__ __forceinline__ int FO(int k, int f, int c) {  // force column f_k[3f+c]
  return 30 * N - 18 + 96 * k + 24 * f + 7 * c;
}
// lane (within the stage row) that owns force / state index psi = 3f + c
__host__ __device__ constexpr int LN(int psi) { return 4 * (psi / 3) + psi % 3; }

// Step-ordered slots of the sweep arrays.  The top chain walks stages 0, 1, ..
// upwards and the bottom chain N-1, N-2, .. downwards; storing the bottom
// stages in reverse (stage k > MID at slot N + MID - k) makes both chains walk
// their slots in the same direction, so every lane of the sweep wave addresses
// step j as (its own base) + j * (a uniform stride): an immediate offset, no
// per-step pointer arithmetic.  SIG: G/H, S^-1 and the right-hand sides
// (stages 0..N-1); SIGX: the state vectors xs[q] = X_q, q = 0..N.
template <int N>
__host__ __device__ constexpr int SIG(int k) { return k <= N / 2 ? k : N + N / 2 - k; }
template <int N>
__host__ __device__ constexpr int SIGX(int q) { return q <= N / 2 ? q : N + N / 2 + 1 - q; }

// Stage rows of the layout: a wave64 holds four 16-lane rows, so the workgroup
// has N rounded up to a multiple of 4 rows.  The rows past N ("phantom" rows)
// run as copies of stage N-1: they read what row N-1 reads and store the same
// values to the same places (identical stores), are left out of the in-place
// updates and the sums, and their maxima duplicate row N-1's.
template <int N>
constexpr int kRows = (N + 3) & ~3;
// Sliced solves (LaunchArgs::slice_iters / resume, mpcq_set_slice) beyond 16 stages: one
// instance per CU there, so a long solve dispatched in a late round ends the launch late
// (DESIGN.md section 8).  Up to 16 stages two instances share a CU and slicing does not
// shorten the modelled launch (section 8b item 9): the code is compiled out and the ADMM
// loop's allocation stays the unsliced one.
// (-DMPCQ_SLICE16: at every horizon -- an experiment)
template <int N>
#ifdef MPCQ_SLICE16
constexpr bool kSlice = true;
#else
constexpr bool kSlice = N > 16;
#endif

// ---------------------------------------------------------------------------
// cross-lane helpers

__device__ __forceinline__ void wave_sync() {
  // LDS is processed in order per wave, so a hand-off inside one wave needs no
  // hardware barrier; the asm memory clobber stops the compiler from moving
  // LDS accesses across this point.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void sync_all() { __syncthreads(); }

template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  // one v_mov_b64_dpp for row_newbcast (DPP64); other controls split in two.
  // Every lane of every row is active wherever these run, so no "old" value.
  return __longlong_as_double(__builtin_amdgcn_mov_dpp(__double_as_longlong(v), CTRL, 0xF, 0xF, false));
}
// broadcast lane J of each 16-lane row (DPP row_newbcast, gfx90a+)
template <int J>
__device__ __forceinline__ double rbc(double v) { return dppd<0x150 + J>(v); }
// broadcast lane J of each quad (quad_perm J,J,J,J)
template <int J>
__device__ __forceinline__ double qbc(double v) { return dppd<85 * J>(v); }

// i0 + sum_{j<12} g_j * v_j, v_j broadcast from lane j of the row (v_fmac_f64_dpp).
// One dependent chain: the fmac issue interval exceeds its latency.  s_nop 1: a VALU
// write of v then a DPP read of it needs two wait states.
__device__ __forceinline__ double bdot12(const double (&g)[12], double v, double i0) {
  double a0 = i0;
  asm volatile("s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %10 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %12 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+v"(a0)
      : "v"(v), "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]), "v"(g[5]), "v"(g[6]), "v"(g[7]),
        "v"(g[8]), "v"(g[9]), "v"(g[10]), "v"(g[11]));
  return a0;
}
// i0 + sum_psi g_psi * v(lane LN(psi)) over a stage's 12 force / state slots, the
// broadcasts folded into v_fmac_f64_dpp (one chain; s_nop 1 covers the DPP read hazard).
__device__ __forceinline__ double bdot_ln12(const double (&g)[12], double v, double i0) {
  double a0 = i0;
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %6 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %7 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %11 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %12 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %13 row_newbcast:14 row_mask:0xf bank_mask:0xf"
      : "+v"(a0)
      : "v"(v), "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]), "v"(g[5]), "v"(g[6]), "v"(g[7]),
        "v"(g[8]), "v"(g[9]), "v"(g[10]), "v"(g[11]));
  return a0;
}
// i0 + sum_{j<6} g_j * v_j, v_j broadcast from lane j of the row: half of a
// 12-term row product (the split sweep, ph_sweep)
__device__ __forceinline__ double bdot6(const double (&g)[6], double v, double i0) {
  double a0 = i0;
  asm volatile("s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf"
      : "+v"(a0)
      : "v"(v), "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]), "v"(g[5]));
  return a0;
}
// i0 + sum_i g_i * v(lane LN(6 + i)), i < 6: the velocity slots
__device__ __forceinline__ double bdot_ln6v(const double (&g)[6], double v, double i0) {
  double a0 = i0;
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %3 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %4 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %5 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %6 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %7 row_newbcast:14 row_mask:0xf bank_mask:0xf"
      : "+v"(a0)
      : "v"(v), "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]), "v"(g[5]));
  return a0;
}
// lower half: keep a; upper half: b of lane l - 32 (one permlane32_swap per dword)
__device__ __forceinline__ double keep_lo_take_lo(double a, double b) {
  const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)y, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
  return __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
}

template <int... J>
__device__ __forceinline__ void gather_seq(double v, double (&all)[12], std::integer_sequence<int, J...>) {
  ((all[J] = rbc<LN(J)>(v)), ...);
}
// the stage's 12-vector from the column lanes
__device__ __forceinline__ void gather12(double v, double (&all)[12]) {
  gather_seq(v, all, std::make_integer_sequence<int, 12>{});
}
template <int... J>
__device__ __forceinline__ void gatherd_seq(double v, double (&all)[12], std::integer_sequence<int, J...>) {
  ((all[J] = rbc<J>(v)), ...);
}
// lanes 0..11 of the row, in lane order
__device__ __forceinline__ void gather_direct12(double v, double (&all)[12]) {
  gatherd_seq(v, all, std::make_integer_sequence<int, 12>{});
}
// sum_j a_j b_j over 12 terms in three interleaved chains (shorter dependency path)
__device__ __forceinline__ double dot12(const double (&a)[12], const double (&b)[12]) {
  double s0 = a[0] * b[0], s1 = a[1] * b[1], s2 = a[2] * b[2];
#pragma unroll
  for (int j = 3; j < 12; j += 3) {
    s0 += a[j] * b[j];
    s1 += a[j + 1] * b[j + 1];
    s2 += a[j + 2] * b[j + 2];
  }
  return (s0 + s1) + s2;
}
// v(lane l) + v(lane l +- 16): rows 0 + 1 and rows 2 + 3, the same sum order in both rows
__device__ __forceinline__ double row_pair_sum(double v) {
  const long long b = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  const double a0 = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
  const double a1 = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
  return a0 + a1;
}
// v(lane l) + v(lane l +- 32): rows 0 + 2 and rows 1 + 3 (one add of the same two values
// in both lanes of a pair: the sum is bit-identical in both)
__device__ __forceinline__ double pair_sum32(double v) {
  const long long b = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  const double a0 = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
  const double a1 = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
  return a0 + a1;
}
// max(a, b) as the hardware instruction, for operands the compiler cannot prove canonical
// (DPP / permlane moves, LDS loads): C's fmax would canonicalize each of them first (see
// clamp_hw); the engine's values are never signalling NaNs
__device__ __forceinline__ double fmax_hw(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double row_pair_max(double v) {
  const long long b = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return fmax_hw(__longlong_as_double(((long long)hi[0] << 32) | lo[0]),
                 __longlong_as_double(((long long)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ double pair_max(double v) {
  const long long b = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return fmax_hw(__longlong_as_double(((long long)hi[0] << 32) | lo[0]),
                 __longlong_as_double(((long long)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// Launder an LDS base pointer: the pointer round-trips a VGPR through an empty asm
// (opaque to the optimiser, so loads through it are not hoisted out of loops)
// and comes back uniform in an SGPR via readfirstlane, costing no VGPR.
template <typename P>
__device__ __forceinline__ void lds_uniform(P*& q) {
  asm volatile("" : "+v"(q));
  if constexpr (sizeof(P*) == 4) {  // an LDS pointer
    q = reinterpret_cast<P*>(static_cast<unsigned long>(
        __builtin_amdgcn_readfirstlane(static_cast<int>(reinterpret_cast<unsigned long>(q)))));
  } else {  // a global-workspace pointer (horizons beyond 32 stages)
    const unsigned long long v = reinterpret_cast<unsigned long long>(q);
    const unsigned lo = __builtin_amdgcn_readfirstlane((int)v), hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    q = reinterpret_cast<P*>(((unsigned long long)hi << 32) | lo);
  }
}
// a wave-uniform double kept in SGPRs
__device__ __forceinline__ double uni(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)bits);
  const int hi = __builtin_amdgcn_readfirstlane((int)(bits >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// min(max(v, lo), hi) as the two hardware instructions.  C's fmax / fmin on values the
// compiler cannot prove canonical (loads, held registers) make it canonicalize each operand
// first (v_max_f64 x, x: IEEE mode quiets a signalling NaN), one extra FP64 instruction per
// bound and use; the engine's values are never signalling NaNs, and for every other input
// (quiet NaNs included: maxNum / minNum) the result is the same.
__device__ __forceinline__ double clamp_hw(double v, double lo, double hi) {
  double r;
  asm("v_max_f64 %0, %1, %2\n\tv_min_f64 %0, %0, %3" : "=&v"(r) : "v"(v), "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ double sel3(int i, double a0, double a1, double a2) {
  return i == 0 ? a0 : (i == 1 ? a1 : a2);
}

// f(integral_constant<int, J>) for J in the sequence, in order
template <typename F, int... J>
__device__ __forceinline__ void for_each_j(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
// a0 += v(lane J) g0, a1 += v(lane J) g1, a2 += v(lane J) g2, v broadcast from lane J of the
// row (v_fmac_f64_dpp; s_nop 1 covers a VALU write of v just before)
template <int J>
__device__ __forceinline__ void fmac3_bc(double& a0, double& a1, double& a2, double v, double g0, double g1, double g2) {
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %3, %4 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %3, %5 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, %3, %6 row_newbcast:%7 row_mask:0xf bank_mask:0xf"
      : "+v"(a0), "+v"(a1), "+v"(a2)
      : "v"(v), "v"(g0), "v"(g1), "v"(g2), "n"(J));
}

// Gauss-Jordan inverse of a 12x12 SPD matrix held one row per column lane
// (row psi in lane LN(psi)); pivots broadcast by row_newbcast, no pivoting.
// gj_fmac<PV>: the pivot's eleven row updates c[j] += a * R[j](lane LN(PV)), j != PV, as
// v_fmac_f64_dpp (the broadcast folded into the FMA: one instruction per entry instead of
// a DPP move and an FMA; fma(a, b, c) and c += b a round alike, so the same bits)
#define MPCQ_GJ11(J)                                                                         \
  asm("s_nop 1\n\t"                                                                          \
      "v_fmac_f64_dpp %0, %11, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %1, %12, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %2, %13, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %3, %14, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %4, %15, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %5, %16, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %6, %17, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %7, %18, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %8, %19, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %9, %20, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %10, %21, %22 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"          \
      : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]), "+v"(o[4]), "+v"(o[5]), "+v"(o[6]),  \
        "+v"(o[7]), "+v"(o[8]), "+v"(o[9]), "+v"(o[10])                                      \
      : "v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7]), \
        "v"(r[8]), "v"(r[9]), "v"(r[10]), "v"(a))
template <int PV>
__device__ __forceinline__ void gj_fmac(double (&c)[12], const double (&R)[12], double a) {
  constexpr int J = LN(PV);
  double o[11], r[11];  // the entries j != PV in order (register renames, no moves)
#pragma unroll
  for (int q = 0; q < 11; ++q) {
    o[q] = c[q < PV ? q : q + 1];
    r[q] = R[q < PV ? q : q + 1];
  }
  if constexpr (J == 0) MPCQ_GJ11(0);
  else if constexpr (J == 1) MPCQ_GJ11(1);
  else if constexpr (J == 2) MPCQ_GJ11(2);
  else if constexpr (J == 4) MPCQ_GJ11(4);
  else if constexpr (J == 5) MPCQ_GJ11(5);
  else if constexpr (J == 6) MPCQ_GJ11(6);
  else if constexpr (J == 8) MPCQ_GJ11(8);
  else if constexpr (J == 9) MPCQ_GJ11(9);
  else if constexpr (J == 10) MPCQ_GJ11(10);
  else if constexpr (J == 12) MPCQ_GJ11(12);
  else if constexpr (J == 13) MPCQ_GJ11(13);
  else if constexpr (J == 14) MPCQ_GJ11(14);
  else static_assert(J < 0, "a column lane LN(i)");
#pragma unroll
  for (int q = 0; q < 11; ++q) c[q < PV ? q : q + 1] = o[q];
}
#undef MPCQ_GJ11
// FOLD = false (beyond 32 stages): the DPP move + FMA form -- the folded blocks hold all
// their operands at once, which the 168 / 128-VGPR budgets there pay for in spills inside
// the ADMM loop (N = 48: 6 -> 15 scratch reloads per iteration in the gfx950 assembly)
// Lazy pivot rows (round 5): the pivot row is not normalised when it is used -- its lane's
// multiplier is 0, so its row stays p and its diagonal becomes 1 -- and each row is scaled
// by its own pivot's 1/d once, after the twelfth step.  A row that has been a pivot is then
// d times the textbook (normalised) row; every later update of it is linear in the row, so
// it stays d times the textbook row, and the final scaling gives the same inverse.  It saves
// the selects that gave the pivot lane a zero base (22 v_cndmask_b32 per pivot, about 40 %
// of the Gauss-Jordan instructions) for 12 multiplies at the end; the rounding differs from
// the normalised form in the last bits.  Up to 32 stages (FOLD); beyond, the normalised
// form stays: the lazy one measured 12-14 % fewer factorisation cycles (N = 16 84.8 k ->
// 74.1 k, N = 32 124 k -> 108 k, profiles/r05h_factime*) with the statuses and iterations
// of the oracle kept, but at N = 48 its (2-3x larger, ~1e-12) first-solve rounding grew to
// 2.1e-7 after five warm-started ticks (8.1e-8 normalised; tools/drift.py,
// profiles/r05j_drift_*).  -DMPCQ_GJ_NORM: the normalised form everywhere.
#ifdef MPCQ_GJ_NORM
template <bool FOLD>
constexpr bool kGjLazy = false;
#else
template <bool FOLD>
constexpr bool kGjLazy = FOLD;
#endif
template <int PV, bool FOLD>
__device__ __forceinline__ void gj_step(double (&R)[12], int me, bool& ok, double& sc) {
  constexpr bool LAZY = kGjLazy<FOLD>;
  const double d = rbc<LN(PV)>(R[PV]);
#ifdef MPCQ_DEBUG_PIVOT
  if (!(d > 0.0) && me == PV) printf("pivot fail blk %d thr %d PV %d d %g\n", (int)blockIdx.x, (int)threadIdx.x, PV, d);
#endif
  if (!(d > 0.0)) ok = false;
  // 1/d: v_rcp_f64 and two Newton steps (the pivots are positive and far from the
  // denormal / overflow range, so the IEEE division's scaling and fix-up are not needed)
  double id = __builtin_amdgcn_rcp(d);
  double e_ = fma(-d, id, 1.0);
  id = fma(id, e_, id);
  e_ = fma(-d, id, 1.0);
  id = fma(id, e_, id);
  // one multiplier per row: every other row R - (R[PV] / d) p, so each entry is a single
  // FMA on the broadcast pivot row; the pivot row itself: p / d (normalised form) or p
  // (lazy: multiplier 0, scaled by sc = 1/d at the end)
  const bool isp = me == PV;
  const double a = isp ? (LAZY ? 0.0 : id) : -(R[PV] * id);
  if constexpr (FOLD) {
    double c[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) c[j] = (isp && !LAZY) ? 0.0 : R[j];
    gj_fmac<PV>(c, R, a);
#pragma unroll
    for (int j = 0; j < 12; ++j)
      if (j != PV) R[j] = c[j];
  } else {
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      if (j == PV) continue;
      const double base = (isp && !LAZY) ? 0.0 : R[j];
      R[j] = fma(a, rbc<LN(PV)>(R[j]), base);
    }
  }
  if constexpr (LAZY) {
    R[PV] = isp ? 1.0 : a;
    if (isp) sc = id;
  } else {
    R[PV] = a;
  }
}
template <bool FOLD, int... P>
__device__ __forceinline__ void gj_seq(double (&R)[12], int me, bool& ok, double& sc, std::integer_sequence<int, P...>) {
  (gj_step<P, FOLD>(R, me, ok, sc), ...);
}
template <bool FOLD>
__device__ __forceinline__ void gj12(double (&R)[12], int me, bool& ok) {
  double sc = 1.0;
  gj_seq<FOLD>(R, me, ok, sc, std::make_integer_sequence<int, 12>{});
  if constexpr (kGjLazy<FOLD>) {
#pragma unroll
    for (int j = 0; j < 12; ++j) R[j] *= sc;
  }
}

// Ro -= G C' for one 12x12 coupling block C held one row per column lane in
// compact form (ca on column CI mod 6, c6 on the velocity columns): column CI of
// the product takes row CI of C from lane LN(CI) by row broadcast
// The broadcasts fold into v_fmac_f64_dpp (one instruction per term instead of a DPP
// move and an FMA); the two chains start from -0 (x + -0 = x for every x, so the first
// term is the plain product, as a multiply) and keep their order: the same bits.
#define MPCQ_SCHUR2_LANE(J)                                                                  \
  asm("s_nop 1\n\t"                                                                          \
      "v_fmac_f64_dpp %0, %2, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"        \
      "v_fmac_f64_dpp %1, %3, %9 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"        \
      "v_fmac_f64_dpp %0, %4, %10 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %1, %5, %11 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %0, %6, %12 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %1, %7, %13 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"       \
      "v_fmac_f64_dpp %0, %14, %15 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"           \
      : "+v"(a0), "+v"(a1)                                                                   \
      : "v"(ca), "v"(c6[0]), "v"(c6[1]), "v"(c6[2]), "v"(c6[3]), "v"(c6[4]), "v"(ga), "v"(G[6]), \
        "v"(G[7]), "v"(G[8]), "v"(G[9]), "v"(G[10]), "v"(c6[5]), "v"(G[11]))
template <int CI, bool FOLD>
__device__ __forceinline__ void schur_col(double (&Ro)[12], const double (&G)[12], double ca,
                                          const double (&c6)[6]) {
  constexpr int J = LN(CI);
  if constexpr (!FOLD) {  // (beyond 32 stages, as gj_step)
    double a0 = G[CI < 6 ? CI : CI - 6] * rbc<J>(ca), a1 = G[6] * rbc<J>(c6[0]);
    a0 = fma(G[7], rbc<J>(c6[1]), a0);
    a1 = fma(G[8], rbc<J>(c6[2]), a1);
    a0 = fma(G[9], rbc<J>(c6[3]), a0);
    a1 = fma(G[10], rbc<J>(c6[4]), a1);
    a0 = fma(G[11], rbc<J>(c6[5]), a0);
    Ro[CI] -= a0 + a1;
    return;
  }
  const double ga = G[CI < 6 ? CI : CI - 6];
  // a0 = ga ca + G7 c1 + G9 c3 + G11 c5, a1 = G6 c0 + G8 c2 + G10 c4 (c broadcast from lane J)
  double a0 = -0.0, a1 = -0.0;
  if constexpr (J == 0) MPCQ_SCHUR2_LANE(0);
  else if constexpr (J == 1) MPCQ_SCHUR2_LANE(1);
  else if constexpr (J == 2) MPCQ_SCHUR2_LANE(2);
  else if constexpr (J == 4) MPCQ_SCHUR2_LANE(4);
  else if constexpr (J == 5) MPCQ_SCHUR2_LANE(5);
  else if constexpr (J == 6) MPCQ_SCHUR2_LANE(6);
  else if constexpr (J == 8) MPCQ_SCHUR2_LANE(8);
  else if constexpr (J == 9) MPCQ_SCHUR2_LANE(9);
  else if constexpr (J == 10) MPCQ_SCHUR2_LANE(10);
  else if constexpr (J == 12) MPCQ_SCHUR2_LANE(12);
  else if constexpr (J == 13) MPCQ_SCHUR2_LANE(13);
  else if constexpr (J == 14) MPCQ_SCHUR2_LANE(14);
  else static_assert(J < 0, "a column lane LN(i)");
  Ro[CI] -= a0 + a1;
}
#undef MPCQ_SCHUR2_LANE
template <bool FOLD, int... C>
__device__ __forceinline__ void schur_cols(double (&Ro)[12], const double (&G)[12], double ca,
                                           const double (&c6)[6], std::integer_sequence<int, C...>) {
  (schur_col<C, FOLD>(Ro, G, ca, c6), ...);
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
// Shared memory of one instance (N=16: 78.6 KB -> 2 instances per CU; N=32:
// 156.7 KB -> 1; N=48: 140 KB with S^{-1} / F W / R^{-1} Q in global memory).

// The sweep matrices (G / H / M^{-1} in GH, S^{-1} in Sm) are 12 x 12, row-major
// with a row stride of RS = 12 doubles (96 B).  Column reads (the outward sweep:
// 12 lanes, consecutive doubles) are conflict-free; the inward sweep's b128 row
// reads (lane r at 96 r) collide 2-3 ways inside a 16-lane group.  A 13-double
// stride removes that but needs 3 KB more LDS than two instances per CU leave at
// N = 16.  GS = one stage's slot.
constexpr int RS = 12, GS = 12 * RS;
// Offset of slot q in GH / Sm: the slots of the bottom chain (q > N/2) sit two
// doubles (16 B) further on.  The sweep's b128 row reads put 4 lanes of one chain
// and 8 of the other in each 16-lane bank group; rows 96 B apart cover only the
// eight 4-bank slots at multiples of 8 dwords, so without the shift the two
// chains' rows met in the same banks (2-way conflicts), with it they interleave.
template <int N>
constexpr int kSlotPad = 2;
template <int N>
__host__ __device__ constexpr int SLOT(int q) { return GS * q + (q > N / 2 ? kSlotPad<N> : 0); }

// Rejected round-4 solve variants (block cyclic reduction of the state system; the
// termination check deferred into the next iteration) were measured slower and removed
// in round 5; their code is kept as a patch, tools/attic/engine_cr_dc_round4.patch, and
// their measurements in DESIGN.md section 8 (round 4) items 3-4.
// Horizons beyond 32 stages do not fit a CU's LDS (N = 48: 236 KB): S^{-1}, F W and
// R^{-1} Q move to a per-instance global workspace (LaunchArgs::work, work_doubles(N)
// doubles per instance, L2-resident), the rest stays in LDS (N = 48: 140 KB).
// Occupancy experiment (round 5, -DMPCQ_OCC16=3 or 4): the 16-stage kernel with the
// beyond-32-stage layout (S^{-1}, R^{-1} Q and the scaled constraint values in the global
// workspace, the split sweep) and __launch_bounds__(..., 3 / 4), so that three or four
// instances share a CU (LDS 39.5 KB; 168 / 128 VGPRs).  Not the default.
#ifdef MPCQ_OCC16
template <int N>
constexpr int kOcc = N == 16 ? MPCQ_OCC16 : 2;
#else
template <int N>
constexpr int kOcc = 2;
#endif
template <int N>
constexpr bool kBig = N > 32 || kOcc<N> > 2;
// F W stays in LDS at every N (the ADMM loop reads it every iteration: from L2 at
// N = 48 it cost the right-hand-side phase ~14 k cycles per iteration, r03d
// stamps); beyond 49 stages the scaled constraint values (126 N - 18 doubles) leave
// LDS instead (N = 64: 197 KB with them, 133 KB without); the engine reads them
// through the same accessors, the stage-parallel phases from L2.
// The nested-dissection state solve (round 6, nd_layout in mpcq_internal.h: N = 32).  The
// state system (block tridiagonal, 12 x 12 blocks) is split at the separator stage s = N/2
// into A = stages 0..s-1 and B = s+1..N-1; each half is factored two-ended on its own, and
// the ADMM loop sweeps A on wave 0 and B on wave 1 at the same time (half the depth of the
// whole-horizon sweep), then solves for the separator's states and corrects both halves by
// the stored spikes W_k = K_A^{-1}[k, s-1] L_s' (k in A) / K_B^{-1}[k, s+1] L_{s+1} (k in B):
//   z = K_A^{-1} b_A, K_B^{-1} b_B      x_s = Sigma^{-1} b_s + P z_{s-1} + Q z_{s+1}
//   x_k = z_k - W_k x_s                 Sigma = D_s - L_s W_{s-1} - L_{s+1}' W_{s+1}
//   P = -Sigma^{-1} L_s, Q = -Sigma^{-1} L_{s+1}'
// The spikes (N x 144 doubles) take the LDS the scaled constraint values leave (they move
// to the workspace, kAbG) with F W at the 72-double stride.
template <int N>
constexpr bool kND = nd_layout(N);
template <int N>
constexpr bool kAbG = N > 49 || kOcc<N> > 2 || kND<N>;
// (kND) the halves: A = stages 0..NDS-1, the separator NDS = N/2, B = NDS+1..N-1 (NDB stages).
// Both halves are swept as NDS-stage systems by one code path: B's sweep carries a phantom
// stage after its last (local stage NDB: zero right-hand side, zero coupling, zero inverse
// slot), which it steps through in parallel with A's real one and which leaves B's solution
// unchanged (its bottom chain starts at the phantom with v = 0).
template <int N> constexpr int NDS = N / 2;
template <int N> constexpr int NDB = N - 1 - N / 2;  // B's real stages (A's: NDS)
// Sweep slots of stage k's right-hand side / w (bo, na, yv) and of its states X_{k+1} (xs).
// Whole-horizon sweep: SIG<N>(k) / SIGX<N>(k+1).  kND: each half in its own step-ordered
// slots (SIG / SIGX of an NDS-stage system), A's first, then B's (B's phantom at
// NDS + SIG<NDS>(NDB)), the separator's last (right-hand side slot N, states slot N+1; B's
// slots start at NDS so that its local X_0 -- the separator, which B's sweep never writes --
// would be A's slot NDS).
template <int N>
__device__ __forceinline__ int RSL(int k) {
  if constexpr (kND<N>) {
    constexpr int S = NDS<N>;
    return k < S ? SIG<S>(k) : (k == S ? N : S + SIG<S>(k - S - 1));
  } else {
    return SIG<N>(k);
  }
}
template <int N>
__device__ __forceinline__ int XSL(int k) {
  if constexpr (kND<N>) {
    constexpr int S = NDS<N>;
    return k < S ? SIGX<S>(k + 1) : (k == S ? N + 1 : S + SIGX<S>(k - S));
  } else {
    return SIGX<N>(k + 1);
  }
}
// (kND) GH / Sm offset of half B's slots: after A's (SLOT<NDS>'s bottom shift included);
// B's phantom's slot (its zero H coupling in GH, its zero inverse in Sm) and right-hand side slot
template <int N> constexpr int kGhB = GS * NDS<N> + 2;
template <int N> constexpr int kPhSlot = kGhB<N> + SLOT<NDS<N>>(SIG<NDS<N>>(NDB<N>));
template <int N> constexpr int kPhRhs = NDS<N> + SIG<NDS<N>>(NDB<N>);
// (kND) stage k's spike block (k != NDS)
template <int N>
__device__ __forceinline__ int WSI(int k) { return k < NDS<N> ? k : k - 1; }
// Beyond 48 stages (13-16 waves: 128 VGPRs) the F_k row is read from the workspace in
// the loop and the z update's constants are batch-loaded from private memory instead
// of being held; from 33 to 48 stages (168 VGPRs) holding them is faster.  Measured at
// every horizon 33..64 with both, either and neither (tools/bigsweep.py,
// profiles/r03o_bigsweep.txt: N = 48 9.05 us per iteration held vs 10.37 not; N = 56
// 19.27 not held vs 20.06).  -DMPCQ_FR_HELD / -DMPCQ_ZC_HELD: held everywhere (experiments).
#ifdef MPCQ_FR_HELD
template <int N> constexpr bool kFrWork = false;
#else
template <int N> constexpr bool kFrWork = N > 48;
#endif
#ifdef MPCQ_ZC_HELD
template <int N> constexpr bool kZcMem = false;
#else
template <int N> constexpr bool kZcMem = N > 48;
#endif
// The outward sweep of ph_sweep_split (33..48 stages) as ph_sweep_lag's: full 12-term
// column products per lane (the outward sweep needs no S^{-1}, which is what sent the
// split sweep's inward half to the stage-parallel S^{-1} phase).  Round 4 (r04h, per
// iteration alone / 256 in flight): N = 40 6.07 -> 5.93 / 6.94 -> 6.73 us, N = 48 6.89 ->
// 6.79 / 7.69 -> 7.62; beyond 48 stages mixed (N = 64 14.96 -> 14.78 / 18.73 -> 19.55), so
// the split products stay there.  -DMPCQ_SPLIT_OUT: the split outward products everywhere.
#ifdef MPCQ_SPLIT_OUT
template <int N> constexpr bool kLagOut = false;
#else
template <int N> constexpr bool kLagOut = N <= 48;
#endif
// Stage stride of F W in LDS (doubles).  ph_recover reads row ph of F_k W_k as three
// ds_read_b128 per lane (16-B units 36 k + 3 ph at a 72-double stride): within each
// 16-lane bank group of that instruction (two stages' lanes), ph 0/1/2 of one stage met
// ph 6/7/8 of the next in the same banks (2-way conflicts); at a 96-double stride (256 B
// x 3, stages 0 mod 16 units apart) the twelve rows of each group land in distinct banks.
// Up to 32 stages, where the LDS has the 24 N doubles (N = 16: 80,048 B, still two
// instances per CU).
template <int N, bool KI = false>
constexpr int kFWS = (!kBig<N> && !KI && !kND<N>) ? 96 : 72;  // (kKI: the LDS goes to Z's columns; kND: to the spikes)
// Up to 16 stages the ADMM loop's exit status goes through LDS (Smem::flag[4]) instead of
// a register carried across the loop: the N = 16 kernel then spills 27 instead of 43
// VGPRs (scratch 256 -> 224 B per lane) and its C2 HBM traffic falls 127 -> 88 MB per
// launch, per-iteration time unchanged (same box, r04u).  At N = 32 the same change made
// the iteration 1.3 % slower and doubled the traffic through the rho-update path's spills,
// so the status stays a register there.
template <int N>
constexpr bool kXstLds = N <= 16;
// From 17 to 48 stages (round 5) the exit status is not carried at all: after the loop it is
// re-derived from what the loop leaves -- a failed factorisation sets sh.flag[2], and an
// early exit stops with iter <= max_iter after the same tests, in the same order, on the
// residuals and infeasibility bits that stay live after the loop anyway.  Carried in a
// register, it was spilled and stored once per check segment at N = 32 (round 4).
// Beyond 48 stages (128 VGPRs) the re-derivation cost the iteration 8 % (N = 64 15.2 -> 16.5
// us alone, 19.7 -> 21.2 at 256 in flight, r05v): there the status is carried as in round 4.
template <int N>
constexpr bool kXstRe = !kXstLds<N> && N <= 48;
// ---- The explicit state-system inverse (kKI, round 5) ------------------------------
// At 16 stages the ADMM loop solves the state system K_s x = r (192 x 192, block
// tridiagonal) with an explicit inverse Z = K_s^{-1} instead of the two-ended sweep: one
// dense matrix-vector product spread over every wave (no serial chain of N/2 dependent
// 12 x 12 steps on one wave).  Z is formed once per factorisation from the sweep's own
// factors (G / H / S^{-1} / M^{-1}): the sweep run on the identity's columns, 16 columns
// at a time as 16 x 16 x 12 products on v_mfma_f64_16x16x4_f64, both chains of a tile in
// one wave.  The workgroup doubles to eight waves (one instance per CU, 256 VGPRs): waves
// 0-3 hold the stages as before, waves 4-7 ("helpers") hold 138 of Z's 192 columns in
// registers (105 doubles per lane); the other 54 columns sit in LDS (KV) and waves 0-3
// multiply them.  The helpers run the stage waves' barrier sequence with no stage work
// (factor / checks with role std::true_type) and take part only in the formation and the
// product.  The oracle's explicit-inverse restatement (full K^{-1} on the C2 and a mixed
// 4096-instance batch) kept statuses and iteration counts identical to its factored solve,
// forces within 1.5e-9.
// Measured and NOT the default (round 5, profiles/r05b_*, r05e_*): parity green on the GPU
// suite (79/79, statuses and iterations = the oracle's), but 1.92 us per iteration alone
// against the sweep's 1.85, and one instance per CU instead of two: C2 86 k, C4 104 k, C5 135 k
// QP/s against 126 k / 222 k / 285 k.  The product is 36,864 FMAs per iteration (ten times
// the sweep's) and its FP64 issue, not a serial chain, then bounds the iteration; the stage
// waves' own instruction stream (right-hand sides, forces, update: ~250 instructions) stays
// on the critical path either way.  Build with -DMPCQ_KINV (make variants compiles it).
#ifdef MPCQ_KINV
template <int N>
constexpr bool kKinv = N == 16;
#else
template <int N>
constexpr bool kKinv = false;
#endif
template <int N, bool SOLVE, bool POLISH>
constexpr bool kKI = kKinv<N> && SOLVE && !POLISH;
template <int N>
struct KinvLay {
  static constexpr int R = 12 * N;             // states (rows / columns of Z)
  static constexpr int KVS = R + 1;            // column stride of KV (odd: conflict-free columns)
  static constexpr int HC = 34;                // helper register columns (per lane: rows l, l+64, l+128)
  static constexpr int SC = 14;                // stage wave LDS columns
  static constexpr int SP0 = 4 * HC, SPC = R - SP0;  // the LDS part: columns 136..191
  // helper h's columns [hc0, hc0 + hcn), stage wave s's [sc0, sc0 + scn)
  __host__ __device__ static constexpr int hc0(int h) { return HC * h; }
  __host__ __device__ static constexpr int hcn(int) { return HC; }
  __host__ __device__ static constexpr int sc0(int s_) { return SP0 + SC * s_; }
  __host__ __device__ static constexpr int scn(int) { return SC; }
  // formation passes: columns [pc0, pc0 + pcn) staged in KV (the last pass is KV's own part)
  static constexpr int NPASS = 4;
  __host__ __device__ static constexpr int pc0(int q) { return q < 3 ? 48 * q : SP0; }
  __host__ __device__ static constexpr int pcn(int q) { return q < 2 ? 48 : (q == 2 ? SP0 - 96 : SPC); }
};
static_assert(KinvLay<16>::hc0(3) + KinvLay<16>::hcn(3) == KinvLay<16>::SP0 &&
                  KinvLay<16>::sc0(3) + KinvLay<16>::scn(3) == KinvLay<16>::R && KinvLay<16>::pcn(3) <= 64 &&
                  KinvLay<16>::pc0(2) + KinvLay<16>::pcn(2) == KinvLay<16>::SP0 && KinvLay<16>::pcn(3) <= 56 &&
                  KinvLay<16>::hc0(3) + 47 < KinvLay<16>::R,
              "Z's column split");
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int N>
struct Work {  // offsets (doubles) inside one instance's workspace
  // SM starts two slots in (a pad kept from round 2; the sweep no longer reads it)
  // FR: each lane's row of F_k (12 doubles, lane-interleaved: entry i of thread t at 16 kRows i + t)
  // (kND: only the zero block and the scaled constraint values)
  static constexpr int SM = 2 * GS, FW = SM + N * GS + 2, QL = FW + 72 * N, ZERO = kND<N> ? 0 : QL + 36 * N, AB = ZERO + 72,
                       FR = AB + (kAbG<N> ? ((126 * N - 18 + 1) & ~1) : 0), SIZE = FR + (N > 48 ? 12 * 16 * kRows<N> : 0);
};

// (kND) the spikes W_k (stage k's 12 x 12 block, row-major; the separator's slot unused) and
// Sigma^{-1}, P, Q of the separator (row-major)
template <int N>
struct NdSmem {
  alignas(16) double Wsp[N - 1][GS];  // stage k's at WSI(k) (the separator has none)
  alignas(16) double Sep[3][GS];
  double Part[3][12];  // the separator's three terms of an iteration (ph_sweep_nd)
};
struct NoNdSmem {};

template <int N, bool KI = false>
struct Smem {
  double Ab[kAbG<N> ? 2 : 126 * N - 18];  // scaled constraint values, CSC order (N > 49: Work<N>::AB)
  // GH[0] = M^{-1}, GH[SIG(k)] = G_k (1 <= k <= m), GH[SIG(k+1)] = H_k (m <= k < N-1),
  // row-major (the sweeps' step order, see SIG).
  // During the factorisation slot k holds Q_k [0,36), F_k W_k [36,108) and the
  // dynamics-row rho of stage k [108,120); during scaling the row factors; in
  // the prologue xref / fsteps / the gait walk.
  alignas(16) double GH[N][GS];
  double GHpad[kND<N> ? 4 : 2];  // the bottom slots' shift (SLOT; kND: both halves')
  // (N > 32: these three live in the global workspace, Work<N>)
  alignas(16) double Sm[kBig<N> ? 1 : N][GS];  // S_k^{-1} / U_k^{-1} of stage k at SLOT(SIG(k)), row-major (row stride RS)
  double Smpad[kND<N> ? 4 : 2];
  // F_k W_k (12x6, row psi at [6 psi]); W_k = B_k' R on rows 6..11: here beyond 32 stages
  // (stage stride 72), FWs at the end up to 32 stages (stride kFWS = 96)
  alignas(16) double FWb[kBig<N> ? N : 1][(kBig<N> || (!KI && !kND<N>)) ? 72 : 2];  // (kKI / kND: no room for the placeholder)
  double QL[kBig<N> ? 1 : N][36];   // B_k F_k W_k = R^{-1} W_k' F_k W_k (6x6)
  union {
    struct {
      // sweep right-hand side of stage k's states = bo[k] + na[k]: bo from stage k
      // itself, na from stage k+1's dynamics rows (Hd (w - beta) + H6 w, summed by
      // ph_rhs); nb is scratch of the checks
      double bo[N + (kND<N> ? 1 : 0)][12];  // (kND: slot N the separator's, RSL)
      double na[N + (kND<N> ? 1 : 0)][12];
      double nb[N][12];
      double yv[N][12];      // w = S^{-1} y of the inward sweep (states / duals during the checks)
      double xs[N + 1 + (kND<N> ? 1 : 0)][12];  // X_k (xs[k+1] = X_{k+1}, stage k's states; kND: sweep slots, XSL)
    } it;
    struct {
      alignas(16) double St[144];  // sweep hand-offs of the factorisation (16-B aligned: the
      alignas(16) double Sb[144];  // couplings read them as column pairs)
      alignas(16) double St2[kND<N> ? 144 : 2];  // (kND) half B's two chains
      alignas(16) double Sb2[kND<N> ? 144 : 2];
    } fa;
  } u;
  // per-wave partial reductions (32 per wave); during the sweeps the sink of lanes
  // whose store is void (lane (t & 31) + 12 j, j <= N/2 + 1)
  double red[(8 * kRows<N> + 32 > 12 * (N / 2 + 2) + 32) ? 8 * kRows<N> + 32 : 12 * (N / 2 + 2) + 32];
  double dump[kND<N> ? 1 : 64];  // sink of predicated stores (never read): lane & 63 (kND: red[], as the sweeps')
  // (13 unused doubles: where round 4's deferred-check arrays sat; they keep every later
  // array's LDS offset, and with it the compiler's register allocation, as measured)
  double pad13_[(KI || kND<N>) ? 1 : 13];
  alignas(16) double zero[72];  // zeros: masked coefficient reads point here instead of selecting
  // flag[4] (kXstLds): the ADMM loop's exit status, written by thread 0 at the (uniform)
  // exits and read by every thread after the loop
  int flag[kXstLds<N> ? 5 : 4];
  // (up to 32 stages) F W at its 96-double stride, last: its round-4 growth leaves every
  // other array's LDS offset -- and the compiler's register allocation -- as before
  alignas(16) double FWs[kBig<N> ? 1 : N][kBig<N> ? 2 : kFWS<N, KI>];
  // (kKI) Z's LDS part, column-major (column c - SP0 at KVS (c - SP0)); during the
  // formation the staging of each pass.  The loop's partial products P[wave][row] sit in GH.
  alignas(16) double KV[KI ? KinvLay<N>::SPC * KinvLay<N>::KVS : 1];
  // (kND) the spikes and the separator's matrices (no room taken at the other horizons)
  [[no_unique_address]] std::conditional_t<kND<N>, NdSmem<N>, NoNdSmem> nd;
};

// prologue aliases inside GH
template <int N>
struct Prologue {
  static constexpr int XR = 0;             // xref, 12(N+1) doubles
  static constexpr int FS = 12 * (N + 1);  // fsteps, 260 doubles
  static constexpr int INTS = FS + 260;    // phase_of_stage[N], contact[20][4] as ints
};

// ---------------------------------------------------------------------------
// The engine kernel.  FUSED: formulate from (xref, fsteps) then solve.
// !FUSED: solve the given (Ax, l, u).  SOLVE=false: formulation only.

template <int N, bool FUSED, bool SOLVE, bool POLISH>
__global__ __launch_bounds__((16 * kRows<N> * (kKI<N, SOLVE, POLISH> ? 2 : 1)), (kKI<N, SOLVE, POLISH> ? 1 : kOcc<N>))
void engine_kernel(mpcq_params p, LaunchArgs a) {
  // KI: the explicit inverse (kKI): twice the threads, waves NW.. are the helpers
  constexpr bool KI = kKI<N, SOLVE, POLISH>;
  constexpr int NR = kRows<N>, NW = NR / 4, T = 16 * NR * (KI ? 2 : 1), n = 24 * N, m = 44 * N, nnz = 126 * N - 18,
                MID = N / 2;
#ifndef MPCQ_STAMP_WAVE
#define MPCQ_STAMP_WAVE 0
#endif
  [[maybe_unused]] constexpr int kStampT = 64 * (MPCQ_STAMP_WAVE < T / 64 ? MPCQ_STAMP_WAVE : T / 64 - 1);
  // the two chains of the state sweeps: top stages 0..MID-1, bottom N-1..MID+1
  // (BOT stages: MID - 1 for even N, MID for odd N), meeting at stage MID
  constexpr int BOT = N - 1 - MID;
  __shared__ Smem<N, KI> sh;
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
  // lane coordinates; the loops launder them (see launder()) so that the
  // compiler recomputes the many LDS offsets derived from them instead of
  // hoisting each one into a register of its own
  const bool phantom = (t >> 4) >= N;  // a row past the horizon: a copy of stage N-1 (kRows)
  int k = phantom ? N - 1 : t >> 4, s = t & 15, f = s >> 2, c = s & 3;
  const bool cl = c < 3;          // column lane (c == 3: friction rows 3, 4 only)
  int cc = cl ? c : 2;            // column component; c == 3 shadows c == 2
  int ph = 3 * f + cc;            // own force / state index in the stage
  if ((int64_t)blockIdx.x >= a.batch) return;
  if constexpr (kSlice<N>) {  // (a resumed slice: its count is on the device, no host round trip)
    if (a.batch_dev && (int64_t)blockIdx.x >= (int64_t)*a.batch_dev) return;
  }
  const int64_t b = a.order ? (int64_t)a.order[blockIdx.x] : (int64_t)blockIdx.x;  // the instance
  STAMP_DECL
  constexpr bool BIG = kBig<N>, ABG = kAbG<N>;
  // the scaled constraint values: LDS, or (N > 49) this instance's workspace (the
  // formulation-only launch builds them straight into its Ax output)
  using acd = std::conditional_t<ABG, g_cd, lds_cd>;
  double* AbW;
  if constexpr (ABG) AbW = SOLVE ? a.work + b * Work<N>::SIZE + Work<N>::AB : a.Ax_out + b * nnz;
  else AbW = sh.Ab;
  acd* Ab = (acd*)AbW;
  lds_cd* GHr = (lds_cd*)&sh.GH[0][0];
  // S^{-1}, R^{-1} Q: LDS, or (N > 32) this instance's global workspace; F W: LDS
  using wcd = std::conditional_t<BIG, g_cd, lds_cd>;
  using wdd = std::conditional_t<BIG, g_d, lds_d>;
  wcd* SmR;
  g_d* FRg = nullptr;  // (kFrWork: N > 48) this lane's F_k row in the workspace, stride 16 kRows
  lds_cd* FWr;
  wcd* QLr;
  wdd* SmW;
  lds_d* FWW;
  wdd* QLW;
  int zFW, zQL;  // offsets of a zero block from FWr / QLr (masked reads)
  if constexpr (BIG) {
    double* const wk = SOLVE ? a.work + b * Work<N>::SIZE : nullptr;  // (formulation only: unused)
    SmW = (wdd*)(wk + Work<N>::SM);
    FWW = (lds_d*)&sh.FWb[0][0];  // (Work<N>::FW stays reserved, unused)
    QLW = (wdd*)(wk + Work<N>::QL);
    if (SOLVE) FRg = (g_d*)(wk + Work<N>::FR + t);
    zFW = (int)(sh.zero - &sh.FWb[0][0]);
    zQL = Work<N>::ZERO - Work<N>::QL;
    if (SOLVE && t < 72) wk[Work<N>::ZERO + t] = 0.0;
  } else {
    if constexpr (ABG) {  // (kND) the zero block the masked coefficient reads of Ab point at
      if (SOLVE && t < 72) a.work[b * Work<N>::SIZE + Work<N>::ZERO + t] = 0.0;
    }
    SmW = (wdd*)&sh.Sm[0][0];
    FWW = (wdd*)&sh.FWs[0][0];
    QLW = (wdd*)&sh.QL[0][0];
    zFW = (int)(sh.zero - &sh.FWs[0][0]);
    zQL = (int)(sh.zero - &sh.QL[0][0]);
  }
  SmR = (wcd*)SmW;
  FWr = (lds_cd*)FWW;
  QLr = (wcd*)QLW;
  double* const gh0 = &sh.GH[0][0];
  int fo = FO<N>(k, f, cc), xo = XO<N>(k, ph);  // own force / state column in Ab
  int cr = (t >> 4) & 1;            // sweep row (wave 0): 0 top-down, 1 bottom-up
  // sweep lane's state index; lanes 12..15 (no state) repeat lanes 0..3, which sit in
  // their bank group, so their reads broadcast instead of conflicting (measured: -2 %
  // per iteration at N <= 16; at N = 32, round 4, same box: SQ_LDS_BANK_CONFLICT per C3
  // launch 1.375e9 -> 0.718e9, 1.57 -> 0.82 of SQ_ACTIVE_INST_LDS, 3.169 -> 3.128 us per
  // iteration, C3 33.85 -> 33.35 ms, profiles/r04e_*; round 2's +2 % there is not
  // reproduced).  Beyond 32 stages (the split sweep) lane 11's row, unmeasured.
  int rr_ = s < 12 ? s : (N <= 32 ? s - 12 : 11);
  // store v at q when c holds, else into this lane's sink (branch-free)
  auto launder = [&]() __attribute__((always_inline)) {
    lds_uniform(Ab); lds_uniform(GHr); lds_uniform(SmR); lds_uniform(FWr); lds_uniform(QLr);
    asm volatile("" : "+v"(k), "+v"(f), "+v"(c), "+v"(cc), "+v"(ph), "+v"(fo), "+v"(xo),
                 "+v"(cr), "+v"(rr_));
  };
  (void)lane;

  // ---- scaled-A accessors ---------------------------------------------------
  auto Xd = [&](int kk, int i) __attribute__((always_inline)) { return Ab[XO<N>(kk, i)]; };
  // dynamics row i of stage kk on X_kk[i] / on X_kk[i+6] (i < 6), kk >= 1
  // (loads stay in bounds for kk == 0 / i >= 6; callers mask those values)
  auto Hd = [&](int kk, int i) __attribute__((always_inline)) {
    return Ab[XO<N>(kk > 0 ? kk - 1 : 0, i) + (i < 6 ? 1 : 2)];
  };
  auto H6 = [&](int kk, int i) __attribute__((always_inline)) {
    return Ab[XO<N>(kk > 0 ? kk - 1 : 0, i < 6 ? i + 6 : 11) + 1];
  };
  // coefficient of force psi = 3fp + cp on dynamics row r (6..11) of stage kk
  auto Bc = [&](int kk, int r, int fp, int cp) __attribute__((always_inline)) -> double {
    const bool nz = r >= 9 || (r >= 6 && cp == r - 6);
    const double v = Ab[FO<N>(kk, fp, cp) + (r >= 9 ? r - 8 : 0)];
    return nz ? v : 0.0;
  };
  // coefficient of force component cp of foot fp on friction row t of that foot
  auto Frc = [&](int kk, int fp, int t_, int cp) __attribute__((always_inline)) -> double {
    const double v = Ab[FO<N>(kk, fp, cp) + (cp == 2 ? 5 + t_ : 5 + (t_ & 1))];
    return (cp == 2 || (t_ < 4 && (t_ >> 1) == cp)) ? v : 0.0;
  };
  // friction row t of foot f at stage k applied to the foot's forces (g0, g1, g2)
  auto fric_row = [&](int t_, double g0, double g1, double g2) __attribute__((always_inline)) {
    const int ta = t_ < 4 ? t_ : 0;
    const double cb = Ab[FO<N>(k, f, 2) + 5 + t_];
    const double ca = Ab[FO<N>(k, f, ta >> 1) + 5 + (ta & 1)];
    const double v = cb * g2;
    return t_ < 4 ? v + ca * ((ta >> 1) == 0 ? g0 : g1) : v;
  };

  // own rows: slot 0 dyn(k, ph) | fric t=3; slot 1 swing(k, ph) | fric t=4; slot 2 fric t=c | none
  auto nat_row = [&](int slot) __attribute__((always_inline)) -> int {
    if (slot == 0) return cl ? 12 * k + ph : 24 * N + 20 * k + 5 * f + 3;
    if (slot == 1) return cl ? 12 * N + 12 * k + ph : 24 * N + 20 * k + 5 * f + 4;
    return cl ? 24 * N + 20 * k + 5 * f + c : -1;
  };
  const int colF = 12 * N + 12 * k + ph, colX = 12 * k + ph;

  // P diagonal of the own columns (MPC.py:255-275)
  const double P0f = p.force_weight;
  double P0X = p.state_weights[0];
#pragma unroll
  for (int e = 1; e < 12; ++e)
    if (ph == e) P0X = p.state_weights[e];

  // Bounds.  FUSED: the dynamics row keeps one value (l = u, MPC.py:410); swing
  // rows are 0 = 0; friction rows u = 0, l = -inf (-OSQP_INFTY) or -fz_max.
  // !FUSED: the caller's l / u for every own row.
  double bnd = 0.0;
  double lo_g[FUSED ? 1 : 3], hi_g[FUSED ? 1 : 3];
  if (t == 0) { sh.flag[0] = 0; sh.flag[1] = 0; sh.flag[2] = 0; sh.flag[3] = 0; }
  for (int e = t; e < 72; e += T) sh.zero[e] = 0.0;  // N = 4: one wave of 64 lanes
  // The sweep arrays start at zero.  No read depends on it (round 3): the steps a
  // sweep chain does not take re-read slots the chain wrote, and stage 0 reads its
  // absent X_0 terms from sh.zero; the zeroing stays as a guard against LDS left
  // over from an earlier workgroup (NaN / Inf).  -DMPCQ_NO_LDS_ZERO builds without
  // it (tools/build_variant.sh nozero ...: the GPU suite must pass on that build).
#ifndef MPCQ_NO_LDS_ZERO
  for (int e = t; e < (int)(sizeof(sh.u.it) / sizeof(double)); e += T) (&sh.u.it.bo[0][0])[e] = 0.0;
#endif

  // ---------------------------------------------------------------- prologue
  if (FUSED || !SOLVE) {
    double* xr = gh0 + Prologue<N>::XR;
    double* fs = gh0 + Prologue<N>::FS;
    int* pos_ = (int*)(gh0 + Prologue<N>::INTS);  // phase_of_stage[N]
    int* con_ = pos_ + N;                         // contact[20][4]
    const double* gx = a.xref + b * 12 * (N + 1);
    const double* gf = a.fsteps + b * 260;
    for (int e = t; e < 12 * (N + 1); e += T) xr[e] = gx[e];
    for (int e = t; e < 260; e += T) fs[e] = gf[e];
    sync_all();
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
        for (int q = 0; q < 4; ++q) {
          const double xv = fs[13 * j + 1 + 3 * q];
          con_[4 * j + q] = !(isnan(xv) || xv == 0.0);
        }
        for (int s_ = 0; s_ < di; ++s_, ++kk)
          if (kk < N) pos_[kk] = j;
      }
      if (kk != N) bad = 1;
      sh.flag[0] = bad ? MPCQ_STATUS_BAD_GAIT : 0;
    }
    sync_all();
    if (sh.flag[0] == 0) {
      for (int e = t; e < 12 * N; e += T) {  // state columns: -I / A (MPC.py:107-115)
        const int kk = e / 12, i = e % 12, xo = XO<N>(kk, i);
        AbW[xo] = -1.0;
        if (kk < N - 1) {
          if (i >= 6) { AbW[xo + 1] = p.dt; AbW[xo + 2] = 1.0; }
          else AbW[xo + 1] = 1.0;
        }
      }
      for (int e = t; e < 4 * N; e += T) {  // foot q of stage kk
        const int kk = e >> 2, q = e & 3;
        const int j = pos_[kk];
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
          lv[r] = ft - xr[r * (N + 1) + kk];
        }
        form_foot(p, xr[5 * (N + 1) + kk], lv[0], lv[1], lv[2], 1.0 - (double)con_[4 * j + q],
                  AbW + FO<N>(kk, q, 0));
      }
      bnd = dyn_bound<N>(p, xr, k, ph);
    }
    if (!SOLVE) {
      sync_all();
      if (t == 0 && a.status) a.status[b] = sh.flag[0];
      if (sh.flag[0] != 0) return;
      double* go = a.Ax_out + b * nnz;
      if constexpr (!ABG)
        for (int e = t; e < nnz; e += T) go[e] = sh.Ab[e];
#pragma unroll
      for (int slot = 0; slot < 3; ++slot) {
        const int r = nat_row(slot);
        if (r < 0) continue;
        double l, u;
        if (cl) {
          if (slot == 0) { l = bnd; u = bnd; }
          else if (slot == 1) { l = 0.0; u = 0.0; }
          else { l = -INFINITY; u = 0.0; }
        } else {
          u = 0.0;
          l = slot == 1 ? -p.fz_max : -INFINITY;  // l[24N+4::5] = -25 (MPC.py:228)
        }
        a.l_out[b * m + r] = l;
        a.u_out[b * m + r] = u;
      }
      return;
    }
  } else {
    const double* ga = a.Ax + b * nnz;
    for (int e = t; e < nnz; e += T) AbW[e] = ga[e];
    if constexpr (!FUSED) {
#pragma unroll
      for (int slot = 0; slot < 3; ++slot) {
        const int r = nat_row(slot);
        lo_g[slot] = r >= 0 ? a.l[b * m + r] : -kInf;
        hi_g[slot] = r >= 0 ? a.u[b * m + r] : kInf;
      }
    }
  }
  if constexpr (SOLVE) {
    sync_all();
    int status = sh.flag[0];
    {  // non-finite data -> NONFINITE (the problem is always feasible otherwise)
      int bad = 0;
      for (int e = t; e < nnz; e += T)
        if (!isfinite(AbW[e])) bad = 1;
      int lgu = 0;  // l > u on an own row (osqp rejects the data)
      if constexpr (FUSED) {
        if (cl && isnan(bnd)) bad = 1;
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (isnan(lo_g[j]) || isnan(hi_g[j])) bad = 1;
          lo_g[j] = lo_g[j] < -kInf ? -kInf : lo_g[j];  // python osqp clamps to +-OSQP_INFTY
          hi_g[j] = hi_g[j] > kInf ? kInf : hi_g[j];
          if (lo_g[j] > hi_g[j]) lgu = 1;
        }
      }
      if (status == 0 && (bad || lgu)) atomicOr(&sh.flag[1], bad ? 1 : 2);
      sync_all();
      if (status == 0 && sh.flag[1]) status = (sh.flag[1] & 1) ? MPCQ_STATUS_NONFINITE : MPCQ_STATUS_BAD_BOUNDS;
    }

    // persistent per-lane state (column values of c == 3 lanes are shadows)
    double xf = 0.0, xX = 0.0, Df = 1.0, DX = 1.0;
    double z[3] = {0.0, 0.0, 0.0}, y[3] = {0.0, 0.0, 0.0}, E[3] = {1.0, 1.0, 1.0};
    double Fr[12];  // row ph of F_k (S_k^{-1} rows live in LDS: sh.Sm)
#pragma unroll
    for (int j = 0; j < 12; ++j) Fr[j] = 0.0;
    unsigned cls = 0u;
    double cscale = 1.0;
    int it_done = 0, n_upd = 0, pol_st = 0, pol_rounds = 0, admm_st = 0;
#ifdef MPCQ_FACTIME
    uint64_t fac_cycles = 0;
#endif
    // (a resumed slice: the rho and the update count it was suspended with)
    double rho_s = kSlice<N> && a.resume ? a.res_rho[b] : (a.rho_in ? a.rho_in[b] : p.rho);
    rho_s = fmin(fmax(rho_s, kRhoMin), kRhoMax);
    if (kSlice<N> && a.resume) n_upd = a.res_i[8 * b + 3];

    // per-row rho / 1/rho from the row's class and the (uniform) rho values
    double r_in = 0.0, r_eq = 0.0, ri_in = 0.0, ri_eq = 0.0;
    double rr[3], ri[3];  // per-row rho and 1/rho (refreshed with rho)
    auto set_rho = [&]() __attribute__((always_inline)) {
      r_in = uni(rho_s);
      r_eq = uni(kRhoEq * rho_s);
      ri_in = uni(1.0 / r_in);
      ri_eq = uni(1.0 / r_eq);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const unsigned cj = (cls >> (2 * j)) & 3u;
        rr[j] = cj == RC_EQ ? r_eq : (cj == RC_INEQ ? r_in : kRhoMin);
        ri[j] = cj == RC_EQ ? ri_eq : (cj == RC_INEQ ? ri_in : 1.0 / kRhoMin);
      }
    };
    auto rho_of_cls = [&](int j) __attribute__((always_inline)) -> double {
      const unsigned cj = (cls >> (2 * j)) & 3u;
      return cj == RC_EQ ? r_eq : (cj == RC_INEQ ? r_in : kRhoMin);
    };
    auto lo_of = [&](int j) __attribute__((always_inline)) -> double {
      if constexpr (FUSED) {
        if (j == 0) return cl ? bnd : -kInf * E[0];
        if (j == 1) return cl ? 0.0 : -p.fz_max * E[1];
        return cl ? -kInf * E[2] : -kInf;
      } else {
        return lo_g[j];
      }
    };
    auto hi_of = [&](int j) __attribute__((always_inline)) -> double {
      if constexpr (FUSED) {
        if (j == 0) return cl ? bnd : 0.0;
        if (j == 1) return 0.0;
        return cl ? 0.0 : kInf;
      } else {
        return hi_g[j];
      }
    };

    // Beyond 48 stages (kZcMem: 128 VGPRs) the ADMM loop spills, and the z / y update's
    // per-row constants (bounds, rho, 1/rho) came back as one scratch reload per use,
    // each waited for before the next.  There they are kept in private memory explicitly
    // and read in one batch per use site (zc_ptr: a laundered pointer, so the loads are
    // neither forwarded nor hoisted).
    using pdbl = __attribute__((address_space(5))) double;
    enum { ZC_LO = 0, ZC_HI = 3, ZC_RR = 6, ZC_RI = 9, ZC_COUNT = 12 };
    double zc_mem_[kZcMem<N> ? ZC_COUNT : 1];
    auto zc_ptr = [&]() __attribute__((always_inline)) -> pdbl* {
      pdbl* q = (pdbl*)&zc_mem_[0];
      asm volatile("" : "+v"(q));
      return q;
    };
    auto zc_store = [&]() __attribute__((always_inline)) {
      if constexpr (kZcMem<N>) {
        pdbl* const q = zc_ptr();
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          q[ZC_LO + j] = lo_of(j);
          q[ZC_HI + j] = hi_of(j);
          q[ZC_RR + j] = rr[j];
          q[ZC_RI + j] = ri[j];
        }
      }
    };

    // ---- row / column operators --------------------------------------------
    // A v for own rows from own forces vf (column lanes), own states vX and the
    // previous stage's states in xs[k]; also returns the force gather.
    auto row_A = [&](double vf, double vX, double (&out)[3]) __attribute__((always_inline)) {
      double fall[12];
      gather12(vf, fall);
      const double* xp = sh.u.it.xs[k];  // xs[0] is never read unmasked
      const double hd = Hd(k, ph), h6 = H6(k, ph);
      const double xa = xp[ph], xb = xp[ph < 6 ? ph + 6 : ph];
      double dyn = Xd(k, ph) * vX;
      const double d1 = dyn + hd * xa;
      const double d2 = d1 + h6 * xb;
      dyn = k >= 1 ? (ph < 6 ? d2 : d1) : dyn;
      double bcf[12];
#pragma unroll
      for (int psi = 0; psi < 12; ++psi) bcf[psi] = Bc(k, ph, psi / 3, psi % 3);
      const double bf = dot12(bcf, fall);
      dyn = ph >= 6 ? dyn + bf : dyn;
      const double g0 = qbc<0>(vf), g1 = qbc<1>(vf), g2 = qbc<2>(vf);
      const double swg = Ab[fo + 4] * vf;
      out[0] = cl ? dyn : fric_row(3, g0, g1, g2);
      out[1] = cl ? swg : fric_row(4, g0, g1, g2);
      out[2] = cl ? fric_row(c, g0, g1, g2) : 0.0;
    };
    auto Pbf = [&]() __attribute__((always_inline)) { return cscale * (Df * P0f * Df); };
    auto PbX = [&]() __attribute__((always_inline)) { return cscale * (DX * P0X * DX); };

    // ---- factorisation --------------------------------------------------------
    // dynamics-row rho of stage kk (published in GH[kk][108..120) at factor time)
    // (stage-keyed scratch: unshifted slots; every read of it precedes the serial
    // steps that overwrite the slots with G / H at SLOT offsets)
    auto rdy = [&](int kk, int i) __attribute__((always_inline)) { return GHr[GS * kk + 108 + i]; };
    auto Qv = [&](int kk, int j1, int j2) __attribute__((always_inline)) { return GHr[GS * kk + 6 * j1 + j2]; };
    // The factorisation's row builders are branch-free: every load is unconditional
    // (indices clamped in range) and the structure is applied by selects.
    // The couplings are sparse: row i of L_kk (and column i) has its nonzeros on
    // column a(i) = i mod 6 and the velocity columns 6..11, so a row is kept as
    // (ca, c6[0..5]).
    // Row i of L_kk (kk >= 1): the dynamics rows of stage kk on (X_{kk+1}[i], X_kk[ci]).
    auto Ctop = [&](int kk, int i, double& ca, double (&c6)[6]) __attribute__((always_inline)) {
      const int iq = i >= 6 ? i - 6 : 0;
      const double ri = rdy(kk, i), xi = Xd(kk, i), hi = Hd(kk, i), h6 = H6(kk, i < 6 ? i : 0);
      const double dv = ri * xi * hi, tv = ri * xi * h6;
      ca = i < 6 ? dv : 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double sc = xi * Qv(kk, iq, j) * Hd(kk, 6 + j);
        const double vv = (6 + j == i ? dv : 0.0) - sc;
        c6[j] = i < 6 ? (j == i ? tv : 0.0) : vv;
      }
    };
    // Column i of L_kk (kk >= 1), i.e. row i of L_kk'.
    auto Cbot = [&](int kk, int i, double& ca, double (&c6)[6]) __attribute__((always_inline)) {
      const int ip = i >= 6 ? i - 6 : 0;
      const double hi = Hd(kk, i);
      const double dv = rdy(kk, i) * Xd(kk, i) * hi;
      const double tv = rdy(kk, ip) * Xd(kk, ip) * H6(kk, ip);
      ca = i < 6 ? dv : tv;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double sc = Xd(kk, 6 + j) * Qv(kk, j, ip) * hi;
        const double vv = (6 + j == i ? dv : 0.0) - sc;
        c6[j] = i >= 6 ? vv : 0.0;
      }
    };
    // Row i of D_kk (the state block of X_{kk+1}).
    auto Drow = [&](int kk, int i, double diag0, double (&Dr)[12]) __attribute__((always_inline)) {
      const bool nx = kk < N - 1;  // stage kk+1 exists
      const int k1 = nx ? kk + 1 : kk;
      const int i6 = i < 6 ? i : i - 6, iq = i >= 6 ? i - 6 : 0;
      const double xi = Xd(kk, i), ri0 = rdy(kk, i);
      const double hi1 = Hd(k1, i), ri1 = rdy(k1, i);
      const double h6p = H6(k1, i6), rp1 = rdy(k1, i6), hp1 = Hd(k1, i6);
      double dg = diag0 + ri0 * xi * xi;
      const double dn = ri1 * hi1 * hi1 + (i >= 6 ? rp1 * h6p * h6p : 0.0);
      dg = nx ? dg + dn : dg;
      const double cross = nx ? (i < 6 ? ri1 * hi1 * h6p : rp1 * hp1 * h6p) : 0.0;
      const int partner = i < 6 ? i + 6 : i - 6;
#pragma unroll
      for (int ci = 0; ci < 12; ++ci) {
        double v = (ci == i) ? dg : 0.0;
        v = (ci == partner) ? cross : v;
        if (ci >= 6) {
          const double s0 = xi * Qv(kk, iq, ci - 6) * Xd(kk, ci);
          const double s1 = hi1 * Qv(k1, iq, ci - 6) * Hd(k1, ci);
          v = i >= 6 ? v - (nx ? s0 + s1 : s0) : v;
        }
        Dr[ci] = v;
      }
    };

      // NS: stages of the system swept (N, or a half of it under kND); RB: its right-hand
      // side (RB[q] + RB[q + RO]), YVB: its y / w slots, XSB: its states, GHB / SMB: its G / H
      // / M^{-1} and S^{-1} slots (ST: the stamp bucket of the wait for the right-hand sides,
      // diagnostic builds).  ND (kND, a half on wave 0 or 1): the caller has passed the barrier
      // that publishes the right-hand sides and runs this on the half's wave only.
      auto ph_sweep_lag = [&](auto ns_tag, auto st_tag, auto nd_tag, lds_cd* const RB, int RO, double* const YVB,
                              double* const XSB, lds_cd* const GHB, lds_cd* const SMB) __attribute__((always_inline)) {
          constexpr int NS = decltype(ns_tag)::value, MID = NS / 2, BOT = NS - 1 - MID;
          [[maybe_unused]] constexpr int ST = decltype(st_tag)::value;
          constexpr bool ND = decltype(nd_tag)::value;
          // P5-P7: the state solve on wave 0 alone (no block barrier inside), up to 32
          // stages (beyond: ph_sweep_split).
          // Inward step j = 1..MID: top kk(j) = j, bottom kk(j) = N-1-j.  Half 0 (rows
          // 0 top / 1 bottom) runs the recurrence y_kk = b_kk - G_kk y_kk(j-1) (G_kk of
          // the top in GH[kk], H_kk of the bottom in GH[kk+1], stored negated), one
          // full 12-term row per lane.  Half 1 (rows 2 / 3) runs the same instruction
          // stream on S^{-1} rows two stages behind: w_kk(j-2) = S^{-1} y_kk(j-2), its y
          // handed over by permlane32_swap.  Step MID+1 is the meeting stage: half 0
          // solves x_m = M^{-1} (y_m + v_m - b_m) (top and bottom rows joined by
          // permlane16_swap), half 1 the last top w.  Then the outward sweeps.
          const int half = (t >> 5) & 1;
#ifndef MPCQ_REP_SWEEP
#define MPCQ_REP_SWEEP 1
#endif
#pragma nounroll
          for (int rep_ = 0; rep_ < MPCQ_REP_SWEEP; ++rep_) {  // > 1: timing experiments only
          double xp = 0.0;
          // Step-ordered bases (SIG): step j's rows / right-hand sides / w / X are at
          // base + j * stride for every lane, an immediate offset.  Half 0: G_j (top,
          // slot j) / H_{N-1-j} (bottom, slot MID+j); half 1: S^{-1} of stage kk(j-2),
          // top slot j-2 / bottom slot MID-1+j.  Step 1's rows are iteration-invariant:
          // wave 0 reads them before the barrier that publishes the right-hand sides.
          // (N > 32: S^{-1} is global, so the row pointer is a generic one)
          using swp = lds_cd;
          using swp2 = lds_cd2;
          swp* const GHs = GHB;
          // (the bottom chain's slots are past N/2: +2, SLOT)
          swp* const Mb = half == 0 ? GHs + (GS * (cr == 0 ? 0 : MID) + (cr == 0 ? 0 : kSlotPad<NS>) + RS * rr_)
                                    : SMB + (GS * (cr == 0 ? -2 : MID - 1) + (cr == 0 ? 0 : kSlotPad<NS>) + RS * rr_);
          double g[12];
          auto row12 = [&](swp* q) __attribute__((always_inline)) {  // 16-B aligned row: 6 ds_read_b128
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              const dbl2 v = ((swp2*)q)[i];
              g[2 * i] = v.x;
              g[2 * i + 1] = v.y;
            }
          };
          // the rows of step j (j a constant after unrolling): every lane reads a slot the
          // factorisation wrote -- the steps a chain does not take (half 1's first step,
          // the bottom chain's steps past its BOT stages at even N) re-read a row of the
          // chain's own, and their products are discarded by the hand-off select / the sink
          auto rowp = [&](int j) __attribute__((always_inline)) -> swp* {
            if (j >= 2 && j <= BOT) return Mb + GS * j;
            const int jj = half == 0 ? (cr == 0 ? j : (j < BOT ? j : BOT))
                                     : (cr == 0 ? (j > 2 ? j : 2) : (j < BOT + 1 ? j : BOT + 1));
            return Mb + GS * jj;
          };
          STAMP(15);  // (diagnostic builds: as in ph_sweep_split)
          if constexpr (ND) {  // (the other waves pass their own barrier: nd_sweep_halves)
            row12(rowp(1));
            sync_all();
          } else {
            if (t < 64) row12(rowp(1));
            sync_all();
          }
          STAMP(ST);
          // outward step j reads G_{MID-j+1}' (top, slot MID+1-j) / H_{MID+j-1}'
          // (bottom, slot N-j) columns: Ob + (MID - j) GS (LDS offsets are unsigned,
          // so the bases sit at the lowest slot a chain reaches)
          lds_cd* const Ob = GHB + (GS * (cr == 0 ? 1 : NS - MID) + (cr == 0 ? 0 : kSlotPad<NS>) + rr_);
          if (ND || t < 64) {
            // the sweeps are every wave's critical path (the other waves of the
            // instance wait at the barrier): issue them ahead of a co-resident
            // instance's stage-parallel phases
            __builtin_amdgcn_s_setprio(3);
            // right-hand side of step j: top stage j (slot j), bottom stage N-1-j (slot
            // MID+1+j, except the meeting stage MID at the bottom's last step BOT, slot
            // MID, which the bottom re-reads in the steps it does not take); na at +12N
            lds_cd* const Bb = RB + (12 * (cr == 0 ? 0 : MID + 1) + rr_);
            lds_cd* const Bm = RB + (12 * MID + rr_);
            auto rhs = [&](int j) __attribute__((always_inline)) -> lds_cd* {  // j: a constant
              return (j >= BOT && cr != 0) ? Bm : Bb + 12 * j;
            };
            // w of stage kk(j-2) (half 1): top slot j-2, bottom slot MID-1+j; the other
            // lanes store into the sink with the same stride
            lds_d* const sink = (lds_d*)&sh.red[0] + (t & 31);
            lds_d* const Yb = (half == 1 && s < 12) ? (lds_d*)YVB + (12 * (cr == 0 ? -2 : MID - 1) + rr_)
                                                    : sink;
            // right-hand sides run two steps ahead: step j sums the one of step j+1
            // (loaded during step j-1) and loads the one of step j+2; half 1 (the w
            // products) starts its chain from 0.  The first two (y_kk(0) and step 1's)
            // are loaded together and waited for once: they were published by the
            // barrier just passed, so this round trip is on the critical path.
            const double m0 = half == 0 ? 1.0 : 0.0;
            double s0 = rhs(0)[0], s1 = rhs(0)[RO];
            double c0 = rhs(1)[0], c1 = rhs(1)[RO];
            asm volatile("" : "+v"(s0), "+v"(s1), "+v"(c0), "+v"(c1));
            double src = half == 0 ? s0 + s1 : 0.0;  // y_kk(0) (half 0)
            double bcn = (c0 + c1) * m0;
            double b0 = rhs(2)[0], b1 = rhs(2)[RO];
#pragma unroll
            for (int j = 1; j <= MID + 1; ++j) {
              asm volatile("" : : : "memory");
              double gc[12];
#pragma unroll
              for (int i = 0; i < 12; ++i) gc[i] = g[i];
              const double bc = j <= MID ? bcn : 0.0;
              if (j < MID) {  // prefetch the next step's rows
                row12(rowp(j + 1));
              } else if (j == MID) {  // the meeting step: M^{-1} rows (half 0), the S walk (half 1)
                row12(half == 0 ? GHs + RS * rr_ : rowp(MID + 1));
                lds_cd* qb = RB + (12 * MID + rr_);
                b0 = qb[0]; b1 = qb[RO];
              } else {  // the last step: the first outward step's columns
#pragma unroll
                for (int i = 0; i < 12; ++i) g[i] = Ob[RS * i + GS * (MID - 1)];
              }
              asm volatile("" : : : "memory");  // the prefetch is issued here, not sunk to its use
              double s_in = src;
              if (j == MID + 1) s_in = half == 0 ? row_pair_sum(src) - (b0 + b1) : src;
              const double acc = bdot12(gc, s_in, bc);
              // the next right-hand side is summed after the chain: its loads were
              // issued at the end of the previous step, and summing them ahead of the
              // chain would put their LDS latency on the critical path
              asm volatile("" : "+v"(b0), "+v"(b1));
              if (j < MID) bcn = (b0 + b1) * m0;
              if (j + 2 <= MID) {
                b0 = rhs(j + 2)[0]; b1 = rhs(j + 2)[RO];
              }
              if (j >= 2 && j <= MID) {  // half 1: w of stage kk(j-2)
                Yb[12 * j] = acc;
              } else if (j == MID + 1) {  // even N: the bottom's kk(MID-1) is the meeting stage (no w)
                if constexpr (NS & 1) Yb[12 * j] = acc;
                else *(cr == 0 ? Yb + 12 * j : sink) = acc;
              }
              if (j <= MID) {
                // half 0 continues with y_kk(j) (the bottom chain stops after step BOT), half 1
                // receives y_kk(j-1) from half 0
                const bool adv = j <= BOT || cr == 0;
                src = keep_lo_take_lo(adv ? acc : src, src);
              } else {
                xp = acc;
                // (lane ids from a laundered thread index: held across the loop, the
                // condition's operand was spilled and its reload waited for here)
                int tl_ = t;
                asm volatile("" : "+v"(tl_));
                if (((tl_ >> 4) & 3) == 0 && (tl_ & 15) < 12) XSB[12 * SIGX<NS>(MID + 1) + (tl_ & 15)] = xp;
              }
            }
            STAMP(6);
          }
          if (ND || t < 64) {
            // Outward step j: top kk = MID-j: X_kk = w_kk - G_{kk+1}' X_{kk+1}; bottom
            // kk = MID+j: X_kk = w_kk - H_{kk-1}' X_{kk-1} (columns from Ob - j GS).  Lane
            // rr reads column rr (a full 12-term product per lane; half 1 repeats half 0).
            // w of stage kk: top slot MID-j, bottom slot N-j (Wb - 12 j); X_kk = xs[kk+1]:
            // top slot MID+1-j, bottom slot N-j (SIGX; Xb - 12 j).  The bottom row's last
            // step (kk = N) is idle: its store goes to the sink.
            // (bases at step MID's slot: step j at base + 12 (MID - j))
            lds_cd* const Wb = (lds_cd*)YVB + (12 * (cr == 0 ? 0 : NS - MID) + rr_);
            lds_d* const sinkO = (lds_d*)&sh.red[0] + (t & 31);
            lds_d* const Xb = (half == 0 && s < 12) ? (lds_d*)XSB + (12 * (cr == 0 ? 1 : NS - MID) + rr_)
                                                    : sinkO;
            wave_sync();  // the w written by half 1
            double bq = Wb[12 * (MID - 1)];
#pragma unroll
            for (int j = 1; j <= MID; ++j) {
              asm volatile("" : : : "memory");
              double gc[12];
#pragma unroll
              for (int i = 0; i < 12; ++i) gc[i] = g[i];
              const double bc = bq;
              if (j < MID) {
#pragma unroll
                for (int i = 0; i < 12; ++i) g[i] = Ob[RS * i + GS * (MID - j - 1)];
                // (even N: the bottom chain has no step MID; it re-reads its last w)
                if (j + 1 <= BOT) bq = Wb[12 * (MID - j - 1)];
                else bq = Wb[12 * (MID - (cr == 0 ? j + 1 : BOT))];
              }
              asm volatile("" : : : "memory");
              const double acc = bdot12(gc, xp, bc);  // x = w - G' x_next with -G stored
              if (j < MID) {
                xp = acc;
                Xb[12 * (MID - j)] = acc;
              } else if constexpr (NS & 1) {
                *Xb = acc;
              } else {  // even N: the bottom chain has no step MID
                *(cr == 0 ? Xb : sinkO) = acc;
              }
            }
            __builtin_amdgcn_s_setprio(0);
          }
          wave_sync();
          }  // MPCQ_REP_SWEEP
      };
      // (kND) Both halves' sweeps, A on wave 0 and B on wave 1, one code path (B as an NDS-stage
      // system with its phantom): the bases differ by a wave-uniform offset.  The barrier that
      // publishes the right-hand sides is inside: the sweep waves read their first rows before
      // theirs (as the whole-horizon sweep does), the other waves pass their own (a wave-uniform
      // branch; every wave executes one s_barrier).
      auto nd_sweep_halves = [&]() __attribute__((always_inline)) {
        if constexpr (kND<N>) {
          constexpr int S = NDS<N>;
          const int wq = __builtin_amdgcn_readfirstlane(t >> 6);
          if (wq < 2) {
            const int o12 = wq ? 12 * S : 0, og = wq ? kGhB<N> : 0;
            ph_sweep_lag(std::integral_constant<int, S>{}, std::integral_constant<int, 3>{}, std::true_type{},
                         (lds_cd*)&sh.u.it.bo[0][0] + o12, 12 * (N + 1), &sh.u.it.yv[0][0] + o12,
                         &sh.u.it.xs[0][0] + o12, GHr + og, (lds_cd*)&sh.Sm[0][0] + og);
          } else {
            sync_all();
          }
        }
      };
    // pr: per-own-row rho override (polish: 1/delta on active rows, 0 elsewhere);
    // nullptr in the ADMM loop, where the class rho applies
    // role: std::false_type for the stage waves; std::true_type (kKI's helper waves) runs the
    // same barrier sequence with no work, so both roles pass every barrier together
    auto factor = [&](auto role, double sigma, const double* pr) __attribute__((always_inline)) -> bool {
      constexpr bool H = decltype(role)::value;
      bool ok = true;
      launder();
      auto rho_of = [&](int j) __attribute__((always_inline)) -> double {
        return pr ? pr[j] : rho_of_cls(j);
      };
      double* gk = gh0 + GS * k;
      if constexpr (!H) {
        if (cl) gk[108 + ph] = rho_of(0);
      }
      sync_all();
      // ---- phase P: F_k = K_ff^{-1} (row ph per column lane), F_k W_k, Q_k
      if constexpr (!H) {
        double rd6[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) rd6[j] = gk[114 + j];
        double rfr[5];
        {
          const double r0 = rho_of(0), r1 = rho_of(1), r2 = rho_of(2);
          rfr[0] = qbc<0>(r2); rfr[1] = qbc<1>(r2); rfr[2] = qbc<2>(r2);
          rfr[3] = qbc<3>(r0); rfr[4] = qbc<3>(r1);
        }
        const double Bo0 = Ab[fo], Bo1 = Ab[fo + 1], Bo2 = Ab[fo + 2], Bo3 = Ab[fo + 3];
        const double sw = Ab[fo + 4];
        const double rsw = rho_of(1);  // swing-row rho (own slot 1)
        double own_fr[5];
#pragma unroll
        for (int t_ = 0; t_ < 5; ++t_) own_fr[t_] = rfr[t_] * Frc(k, f, t_, cc);
        const double dgf = Pbf() + sigma + rsw * sw * sw;
#pragma unroll
        for (int psi = 0; psi < 12; ++psi) {
          const int fp = psi / 3, cp = psi % 3;
          double v = (cp == cc) ? rd6[cp] * Bo0 * Ab[FO<N>(k, fp, cp)] : 0.0;
          v += rd6[3] * Bo1 * Ab[FO<N>(k, fp, cp) + 1];
          v += rd6[4] * Bo2 * Ab[FO<N>(k, fp, cp) + 2];
          v += rd6[5] * Bo3 * Ab[FO<N>(k, fp, cp) + 3];
          if (psi == ph) v += dgf;
          if (fp == f) {
            double fr = 0.0;
#pragma unroll
            for (int t_ = 0; t_ < 5; ++t_) fr += own_fr[t_] * Frc(k, f, t_, cp);
            v += fr;
          }
          Fr[psi] = v;
        }
        gj12<!kBig<N>>(Fr, ph, ok);
        if constexpr (kFrWork<N>) {
#pragma unroll
          for (int i = 0; i < 12; ++i) FRg[16 * NR * i] = Fr[i];
        }
        // F W (row ph): W[psi][j] = rho_{6+j} B[6+j][psi]
        double fw[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          double acc = 0.0;
#pragma unroll
          for (int psi = 0; psi < 12; ++psi) {
            const double bv = Bc(k, 6 + j, psi / 3, psi % 3);
            if (j >= 3 || psi % 3 == j) acc += Fr[psi] * (rd6[j] * bv);
          }
          fw[j] = acc;
        }
        if (cl) {
#pragma unroll
          for (int j = 0; j < 6; ++j) { gk[36 + 6 * ph + j] = fw[j]; FWW[kFWS<N, KI> * k + 6 * ph + j] = fw[j]; }
        }
        wave_sync();
        // Q = W' (F W): 36 entries over the row's 16 lanes
        for (int e = s; e < 36; e += 16) {
          const int j1 = e / 6, j2 = e % 6;
          const double r1 = gk[114 + j1];
          double acc = 0.0;
#pragma unroll
          for (int psi = 0; psi < 12; ++psi)
            acc += (r1 * Bc(k, 6 + j1, psi / 3, psi % 3)) * gk[36 + 6 * psi + j2];
          gk[e] = acc;
          QLW[36 * k + e] = acc / r1;
        }
      }
      const double dgX = PbX() + sigma;
      sync_all();
      STAMP(13);
      // ---- phase S: two-ended block factorisation of the state system.  Per
      // step the active row keeps one 12-vector live (its row of S / U / M):
      // L goes to LDS entry by entry, G / H straight to their GH slot.
      double* const St = sh.u.fa.St;
      double* const Sb = sh.u.fa.Sb;
      // Step j < MID: top row k = j (C = L_k against S_{k-1}^{-1}) and bottom row
      // k = N-1-j > MID (C = L_{k+1}' against U_{k+1}^{-1}) in parallel; step MID:
      // the meeting row (both couplings).  G_k -> GH[k], H_k -> GH[k+1], M^{-1} -> GH[0].
      // One coupling of the active row: upper C = L_k (row ph) against S_{k-1}^{-1}
      // (St), giving G_k -> GH[k]; lower C = L_{k+1}' (row ph) against U_{k+1}^{-1}
      // (Sb), giving H_k -> GH[k+1].  Ro -= (C S^{-1}) C'.  Products run block by
      // block (a compiler fence per block keeps the loads from piling up).
      // Every row's D / L coefficients depend only on its own stage and the next
      // one, all final here: each lane builds its rows before the serial steps
      // (in parallel, one LDS round trip) instead of inside them.
      double Dr0[12], cta, ct6[6], cba, cb6[6];
      Drow(k, ph, dgX, Dr0);
      Ctop(k, ph, cta, ct6);                      // used from k >= 1 only
      Cbot(k < N - 1 ? k + 1 : k, ph, cba, cb6);  // used from k < N-1 only
      auto couple = [&](bool upper, double (&Ro)[12]) __attribute__((always_inline)) {
        const double ca = upper ? cta : cba;
        double c6[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) c6[j] = upper ? ct6[j] : cb6[j];
        const double* const Sp = upper ? St : Sb;
        wave_sync();  // this row's reads of GH[k], GH[k+1] are done
        const int ar = ph < 6 ? ph : ph - 6;
        // two columns at a time: their fourteen operands as seven 16-B reads, loaded
        // together and waited for once, and two independent FMA chains (each column's
        // sum in the same order as one at a time; row blocks waited load by load under
        // the register pressure here)
        double G[12];
        if constexpr (kBig<N>) {  // (beyond 32 stages one column at a time, as gj_step)
#pragma unroll
          for (int ci = 0; ci < 12; ++ci) {
            double sv[7];
            sv[0] = Sp[12 * ar + ci];
#pragma unroll
            for (int j = 0; j < 6; ++j) sv[1 + j] = Sp[12 * (6 + j) + ci];
            double gv = ca * sv[0];
#pragma unroll
            for (int j = 0; j < 6; ++j) gv = fma(c6[j], sv[1 + j], gv);
            G[ci] = gv;
            asm volatile("" ::: "memory");
          }
        } else {
#pragma unroll
        for (int ci = 0; ci < 12; ci += 2) {
          const dbl2 s0 = *(lds_cd2*)(Sp + 12 * ar + ci);
          dbl2 su[6];
#pragma unroll
          for (int j = 0; j < 6; ++j) su[j] = *(lds_cd2*)(Sp + 12 * (6 + j) + ci);
          double g0 = ca * s0.x, g1 = ca * s0.y;
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            g0 = fma(c6[j], su[j].x, g0);
            g1 = fma(c6[j], su[j].y, g1);
          }
          G[ci] = g0;
          G[ci + 1] = g1;
          asm volatile("" ::: "memory");
        }
        }
        if (cl) {
          double* const Gd = gh0 + SLOT<N>(upper ? SIG<N>(k) : SIG<N>(k + 1)) + RS * ph;
#pragma unroll
          for (int ci = 0; ci < 12; ++ci) Gd[ci] = -G[ci];  // stored negated
        }
        schur_cols<!kBig<N>>(Ro, G, ca, c6, std::make_integer_sequence<int, 12>{});
      };
      if constexpr (kND<N>) {
        // (kND) Two two-ended factorisations, one per half, their steps interleaved (step j of
        // both; B's meeting comes one step before A's at N = 32).  Half A's rows: stages
        // 0..S-1, its top chain from stage 0, its bottom chain from S-1 (no coupling to the
        // separator); half B's: S+1..N-1, its top chain from S+1 (no coupling to the separator).
        // G / H / M^{-1} / S^{-1} in the half's slots (SLOT<NS>(SIG<NS>(local stage)), B's at
        // kGhB); the chains hand off through St / Sb (A) and St2 / Sb2 (B).
        constexpr int S = NDS<N>, NB = NDB<N>, MID2 = S / 2;
        static_assert(S >= 4 && NB >= 3 && NB <= S, "the halves of the nested-dissection solve");
        const int hh = k < S ? 0 : (k > S ? 1 : 2);  // 0: A, 1: B, 2: the separator
        const int kl = hh == 0 ? k : k - S - 1;        // stage in the half
        const int nreal = hh == 0 ? S : NB;            // (B's local stage NB is its phantom)
        double* const Sth = hh == 0 ? St : sh.u.fa.St2;
        double* const Sbh = hh == 0 ? Sb : sh.u.fa.Sb2;
        const int hb = hh == 0 ? 0 : kGhB<N>;
        auto hslot = [&](int q) __attribute__((always_inline)) -> int { return hb + SLOT<S>(SIG<S>(q)); };
        // couple(): C S^{-1} from the given hand-off, G / H into the given slot row
        auto couple_nd = [&](bool upper, double (&Ro)[12], const double* Sp, double* Gd)
            __attribute__((always_inline)) {
          const double ca = upper ? cta : cba;
          double c6[6];
#pragma unroll
          for (int j = 0; j < 6; ++j) c6[j] = upper ? ct6[j] : cb6[j];
          wave_sync();  // this row's reads of its G / H slots are done
          const int ar = ph < 6 ? ph : ph - 6;
          double G[12];
#pragma unroll
          for (int ci = 0; ci < 12; ci += 2) {
            const dbl2 s0 = *(lds_cd2*)(Sp + 12 * ar + ci);
            dbl2 su[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) su[j] = *(lds_cd2*)(Sp + 12 * (6 + j) + ci);
            double g0 = ca * s0.x, g1 = ca * s0.y;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
              g0 = fma(c6[j], su[j].x, g0);
              g1 = fma(c6[j], su[j].y, g1);
            }
            G[ci] = g0;
            G[ci + 1] = g1;
            asm volatile("" ::: "memory");
          }
          if (cl) {
#pragma unroll
            for (int ci = 0; ci < 12; ++ci) Gd[ci] = -G[ci];  // stored negated
          }
          schur_cols<true>(Ro, G, ca, c6, std::make_integer_sequence<int, 12>{});
        };
        // B's phantom: zero coupling (its G / H slot) and zero inverse (its S^{-1} slot), once the
        // stage-keyed factor scratch in GH (Q_k, F_k W_k, rho) has been read (Drow / Ctop / Cbot)
        sync_all();
        for (int e = t; e < GS; e += T) {
          gh0[kPhSlot<N> + e] = 0.0;
          SmW[kPhSlot<N> + e] = 0.0;
        }
#pragma nounroll
        for (int j = 0; j <= MID2; ++j) {
          launder();
          const bool act = hh < 2;
          const bool top = act && j < MID2 && kl == j;
          const bool bot = act && j < MID2 && kl == S - 1 - j && kl > MID2;
          const bool mrow = act && j == MID2 && kl == MID2;
          if (!H && (top || bot || mrow)) {
            const bool useT = (top && kl > 0) || mrow, useB = (bot && kl < nreal - 1) || mrow;
            double Ro[12];
#pragma unroll
            for (int ci = 0; ci < 12; ++ci) Ro[ci] = Dr0[ci];
            if (useT) couple_nd(true, Ro, Sth, gh0 + hslot(kl) + RS * ph);
            if (useB) couple_nd(false, Ro, Sbh, gh0 + hslot(kl + 1) + RS * ph);
            gj12<true>(Ro, ph, ok);
            if (cl) {
#pragma unroll
              for (int ci = 0; ci < 12; ++ci) SmW[hslot(kl) + RS * ph + ci] = Ro[ci];
            }
            wave_sync();  // the previous inverse has been consumed by this row
            if (cl) {
              double* dst = mrow ? gh0 + hb + RS * ph : (bot ? Sbh : Sth) + 12 * ph;
#pragma unroll
              for (int ci = 0; ci < 12; ++ci) dst[ci] = Ro[ci];
            }
          }
          sync_all();
        }
        // The spikes: each half solved with its coupling to the separator as the right-hand
        // side, one column at a time through the ADMM loop's own half sweeps -- A with column
        // cI of L_s' at stage S-1 (row ph of L_s' is stage S-1's lower coupling row, cba /
        // cb6), B with column cI of L_{S+1} at stage S+1 (its upper coupling row, cta / ct6);
        // W_k = the solution's block at stage k.  (u.fa's hand-offs are dead: u.it's right-hand
        // sides, w and states take their place.)
        {
          const int ar = ph < 6 ? ph : ph - 6;
#pragma nounroll
          for (int cI = 0; cI < 12; ++cI) {
            launder();
            const bool lo = k == S - 1, up = k == S + 1;
            double ca = lo ? cba : cta, cv = 0.0;
#pragma unroll
            for (int j = 0; j < 6; ++j)
              if (cI == 6 + j) cv = lo ? cb6[j] : ct6[j];
            const double rv = (lo || up) ? (cI == ar ? ca : 0.0) + cv : 0.0;
            if (cl) {
              sh.u.it.bo[RSL<N>(k)][ph] = rv;
              sh.u.it.na[RSL<N>(k)][ph] = 0.0;
              if (k == S) { sh.u.it.bo[kPhRhs<N>][ph] = 0.0; sh.u.it.na[kPhRhs<N>][ph] = 0.0; }
            }
            nd_sweep_halves();  // (its barrier publishes the right-hand sides)
            sync_all();
            if (cl && k != S) sh.nd.Wsp[WSI<N>(k)][RS * ph + cI] = sh.u.it.xs[XSL<N>(k)][ph];
          }
        }
        sync_all();
        // The separator: Sigma = D_S - L_S W_{S-1} - L_{S+1}' W_{S+1} (row ph: stage S's upper
        // coupling row cta / ct6 against W_{S-1}, its lower one cba / cb6 against W_{S+1}), its
        // inverse, P = -Sigma^{-1} L_S and Q = -Sigma^{-1} L_{S+1}' (rows of L_S / L_{S+1}' from
        // the row's lanes by broadcast).
        if (k == S) {
          const int ar = ph < 6 ? ph : ph - 6;
          double Ro[12];
#pragma unroll
          for (int ci = 0; ci < 12; ++ci) {
            const double* const Wa = &sh.nd.Wsp[WSI<N>(S - 1)][0];
            const double* const Wb = &sh.nd.Wsp[WSI<N>(S + 1)][0];
            double ga = cta * Wa[12 * ar + ci], gb = cba * Wb[12 * ar + ci];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
              ga = fma(ct6[j], Wa[12 * (6 + j) + ci], ga);
              gb = fma(cb6[j], Wb[12 * (6 + j) + ci], gb);
            }
            Ro[ci] = Dr0[ci] - ga - gb;
          }
          gj12<true>(Ro, ph, ok);
          double Pr[12], Qr[12];
#pragma unroll
          for (int c = 0; c < 12; ++c) {
            const double lt = (c == ar ? cta : 0.0) + (c >= 6 ? ct6[c >= 6 ? c - 6 : 0] : 0.0);
            const double lb = (c == ar ? cba : 0.0) + (c >= 6 ? cb6[c >= 6 ? c - 6 : 0] : 0.0);
            Pr[c] = -bdot_ln12(Ro, lt, 0.0);
            Qr[c] = -bdot_ln12(Ro, lb, 0.0);
          }
          if (cl) {
#pragma unroll
            for (int ci = 0; ci < 12; ++ci) {
              sh.nd.Sep[0][RS * ph + ci] = Ro[ci];
              sh.nd.Sep[1][RS * ph + ci] = Pr[ci];
              sh.nd.Sep[2][RS * ph + ci] = Qr[ci];
            }
          }
        }
        sync_all();
      } else {
      // Step j < MID: top row k = j and bottom row k = N-1-j > MID in parallel; step
      // MID: the meeting row (both couplings).  M^{-1} -> GH[0].
#pragma nounroll
      for (int j = 0; j <= MID; ++j) {
        launder();
        const bool mid = j == MID;
        const bool top = !mid && k == j, bot = !mid && k == N - 1 - j && k > MID, mrow = mid && k == MID;
        if (!H && (top || bot || mrow)) {
          const bool useT = (top && k > 0) || mrow, useB = (bot && k < N - 1) || mrow;
          double Ro[12];
#pragma unroll
          for (int ci = 0; ci < 12; ++ci) Ro[ci] = Dr0[ci];
          if (useT) couple(true, Ro);
          if (useB) couple(false, Ro);
          gj12<!kBig<N>>(Ro, ph, ok);
          if (cl) {
#pragma unroll
            for (int ci = 0; ci < 12; ++ci) SmW[SLOT<N>(SIG<N>(k)) + RS * ph + ci] = Ro[ci];
          }
          wave_sync();  // the previous inverse has been consumed by this row
          if (cl) {
            double* dst = mrow ? &sh.GH[0][RS * ph] : (bot ? Sb : St) + 12 * ph;
#pragma unroll
            for (int ci = 0; ci < 12; ++ci) dst[ci] = Ro[ci];
          }
        }
        sync_all();
      }
      }  // kND
      STAMP(14);
      // a non-positive pivot anywhere fails the whole instance (uniform result)
      if (!ok) atomicOr(&sh.flag[2], 1);
      sync_all();
      const bool good = sh.flag[2] == 0;
      sync_all();
      return good;
    };

    // ---- residuals (OSQP update_info), uniform results ---------------------
    double pri_res = 0.0, dua_res = 0.0, eps_pri = 0.0, eps_dua = 0.0, s_pri = 0.0, s_dua = 0.0;
  // per-lane constants of the ADMM loop and the residuals: LDS offsets, flags
    const bool hp = k >= 1, isv = ph >= 6;
    const int zXS = (int)(sh.zero - &sh.u.it.xs[0][0]);  // X_0 is not stored: stage 0 reads zeros
    const double m2 = cc == 2 ? 1.0 : 0.0;
    // masked variants for the loop: a lane whose term is structurally absent reads a
    // zero (stage 0 has no previous stage; H6 only on the position rows; the force Schur
    // terms beta, (R^-1 Q) g only on the velocity rows), so no selects are needed
    int zAb;  // offset of a zero block from Ab (masked reads)
    if constexpr (ABG) zAb = Work<N>::ZERO - Work<N>::AB;
    else zAb = (int)(sh.zero - sh.Ab);
    lds_cd* XSr = (lds_cd*)&sh.u.it.xs[0][0];
    double* const Wdump = kND<N> ? &sh.red[t & 63] : &sh.dump[t & 63];  // (red: no reduction is live in ph_rhs)
    // The LDS offsets of the lane's coefficients, derived from its coordinates.  O0
    // is derived once and held (the loop phases up to 32 stages, where the ADMM loop
    // has the registers); a phase run between long stretches of other work -- the
    // termination check at every N, every loop phase beyond 32 stages (168 VGPRs) --
    // re-derives them from freshly laundered coordinates (MPCQ_LANE_OFFS(true)), a
    // few integer ops each: held across the ADMM loop, the compiler spills them, and
    // each use then waits on its own scratch round trip (the reloads sit right in
    // front of their LDS reads, one after another).
    struct LaneOffs {
      int oXd, oHd, oH6, oF, oFa, oFb, oF4, oFW, oQL, oXSp, oXSp6, rXS, rXSpm, rXSp6m, oHdm, oH6m, oFWcm, oQLm,
          oB0;
      bool ta0;
      double* Wbo;
      double* Wna;
    };
    auto offs = [&]() __attribute__((always_inline)) -> LaneOffs {
      const bool hp_ = k >= 1, isv_ = ph >= 6;
      LaneOffs o;
      o.oXd = xo;                                                 // Xd(k, ph)
      o.oHd = XO<N>(hp_ ? k - 1 : 0, ph) + (ph < 6 ? 1 : 2);      // Hd(k, ph)
      o.oH6 = XO<N>(hp_ ? k - 1 : 0, ph < 6 ? ph + 6 : 11) + 1;   // H6(k, ph)
      o.oF = fo;
      const int ta = c < 3 ? c : 3;  // first own friction row
      o.ta0 = (ta >> 1) == 0;
      o.oFa = FO<N>(k, f, ta >> 1) + 5 + (ta & 1);
      o.oFb = FO<N>(k, f, 2) + 5 + ta;
      o.oF4 = FO<N>(k, f, 2) + 9;
      o.oFW = kFWS<N, KI> * k + 6 * ph;
      const int oFWc = kFWS<N, KI> * k + (isv_ ? ph - 6 : 0);
      o.oQL = 36 * k + 6 * (isv_ ? ph - 6 : 0);
      o.oXSp = 12 * k + ph;  // natural order (update_info)
      o.oXSp6 = 12 * k + (ph < 6 ? ph + 6 : ph);
      // the sweep's states in its slots (SIGX): own X_{k+1}, the previous stage's X_k
      auto xsl = [](int kk) __attribute__((always_inline)) -> int { return 12 * XSL<N>(kk); };
      o.rXS = xsl(k) + ph;
      o.rXSpm = hp_ ? xsl(k - 1) + ph : zXS;
      o.rXSp6m = hp_ ? xsl(k - 1) + (ph < 6 ? ph + 6 : ph) : zXS;
      o.oHdm = hp_ ? o.oHd : zAb;
      o.oH6m = hp_ && !isv_ ? o.oH6 : zAb;
      o.oFWcm = isv_ ? oFWc : zFW;
      o.oQLm = isv_ ? o.oQL : zQL;
      o.oB0 = FO<N>(k, 0, 0) + (ph >= 9 ? ph - 8 : 0);  // B row ph on force (fp, cp): + 24 fp + 7 cp
      if constexpr (KI) {  // natural stage order: the product reads them by state index
        o.Wbo = &sh.u.it.bo[k][ph];
        o.Wna = &sh.u.it.na[hp_ ? k - 1 : N - 1][ph];
      } else {
        o.Wbo = &sh.u.it.bo[RSL<N>(k)][ph];
        o.Wna = &sh.u.it.na[RSL<N>(hp_ ? k - 1 : N - 1)][ph];
      }
      return o;
    };
    const LaneOffs O0 = offs();
#define MPCQ_LANE_OFFS(RECOMP)                                                                              \
  if constexpr (RECOMP) launder();                                                                         \
  const LaneOffs O_ = (RECOMP) ? offs() : O0;                                                              \
  [[maybe_unused]] const int oXd = O_.oXd, oHd = O_.oHd, oH6 = O_.oH6, oF = O_.oF, oFa = O_.oFa,           \
                             oFb = O_.oFb, oF4 = O_.oF4, oFW = O_.oFW, oQL = O_.oQL, oXSp = O_.oXSp,       \
                             oXSp6 = O_.oXSp6, rXS = O_.rXS, rXSpm = O_.rXSpm, rXSp6m = O_.rXSp6m,         \
                             oHdm = O_.oHdm, oH6m = O_.oH6m, oFWcm = O_.oFWcm, oQLm = O_.oQLm, oB0 = O_.oB0; \
  [[maybe_unused]] const bool ta0 = O_.ta0;                                                                \
  [[maybe_unused]] double* const Wbo = O_.Wbo;                                                             \
  [[maybe_unused]] double* const Wna = O_.Wna
    // beyond 32 stages the loop phases re-derive them too
    constexpr bool kRecompLoop = BIG || KI;  // (kKI: the helpers' registers set the budget)
    auto launder_p = [&]() __attribute__((always_inline)) {
      lds_uniform(Ab); lds_uniform(GHr); lds_uniform(SmR); lds_uniform(FWr); lds_uniform(QLr); lds_uniform(XSr);
    };
    // force column of A' v for own-row values v (dynamics rows 6..11 by row broadcast,
    // swing, friction by quad broadcast)
    auto colF_c = [&](const double (&A)[10], const double (&v)[3]) __attribute__((always_inline)) -> double {
      const double w6 = rbc<LN(6)>(v[0]), w7 = rbc<LN(7)>(v[0]), w8 = rbc<LN(8)>(v[0]);
      const double w9 = rbc<LN(9)>(v[0]), w10 = rbc<LN(10)>(v[0]), w11 = rbc<LN(11)>(v[0]);
      const double wf0 = qbc<0>(v[2]), wf1 = qbc<1>(v[2]), wf2 = qbc<2>(v[2]);
      const double wf3 = qbc<3>(v[0]), wf4 = qbc<3>(v[1]);
      double sA = A[0] * (cc == 0 ? w6 : (cc == 1 ? w7 : w8));
      double sB = A[1] * w9;
      sA += A[2] * w10;
      sB += A[3] * w11;
      sA += A[4] * v[1];
      sB += A[5] * (cc == 1 ? wf2 : wf0);
      sA += A[6] * (cc == 1 ? wf3 : wf1);
      const double sC = (A[7] * wf2 + A[8] * wf3) + A[9] * wf4;  // friction rows 2..4 (cc == 2)
      return (sA + sB) + m2 * sC;
    };
    auto colF_off = [&](const double (&v)[3]) __attribute__((always_inline)) -> double {
      double A[10];
#pragma unroll
      for (int i = 0; i < 10; ++i) A[i] = Ab[fo + i];
      return colF_c(A, v);
    };
    // Row maxima of several quantities at once, by a transposing butterfly over the
    // 16-lane row: each step pairs lane s with a partner that differs in one bit
    // (row_mirror: s ^ 15, bit 3; row_half_mirror: s ^ 7, bit 2; quad xor 2, bit 1;
    // quad xor 1, bit 0) and the lanes on either side of that bit keep half of the
    // quantities, so a step reduces half as many values as the one before instead of
    // every quantity taking all four steps (12 quantities: 13 maxima and 13 DPP moves
    // instead of 48 each, for 26 two-way selects instead of 12).  Maxima are exact in
    // any order: the results are the ones the per-quantity reduction gave.
    // one step: lanes with the bit clear keep quantity a, the others b
    auto tstep = [](auto ctrl, double a, double b, bool hi) __attribute__((always_inline)) {
      constexpr int C = decltype(ctrl)::value;
      const double mine = hi ? b : a, send = hi ? a : b;
      return fmax_hw(mine, dppd<C>(send));
    };
    auto sstep = [](auto ctrl, double a) __attribute__((always_inline)) {
      constexpr int C = decltype(ctrl)::value;
      return fmax_hw(a, dppd<C>(a));
    };
    using kMirror = std::integral_constant<int, 0x140>;   // row_mirror (s ^ 15)
    using kHalfMir = std::integral_constant<int, 0x141>;  // row_half_mirror (s ^ 7)
    using kXor2 = std::integral_constant<int, 0x4E>;      // quad_perm [2,3,0,1]
    using kXor1 = std::integral_constant<int, 0xB1>;      // quad_perm [1,0,3,2]
    // six quantities over bits 3, 2, 1: lane s keeps quantity 3 b3 + (b2 ? 2 : b1),
    // maximised over the eight lanes s ^ {0, 15, 7, 8, 2, 13, 5, 10}
    auto tred6 = [&](const double (&v)[6], int s_) __attribute__((always_inline)) {
      const bool h3 = s_ & 8, h2 = s_ & 4, h1 = s_ & 2;
      const double a0 = tstep(kMirror{}, v[0], v[3], h3), a1 = tstep(kMirror{}, v[1], v[4], h3),
                   a2 = tstep(kMirror{}, v[2], v[5], h3);
      const double c0 = tstep(kHalfMir{}, a0, a2, h2), c1 = tstep(kHalfMir{}, a1, a2, h2);
      return tstep(kXor2{}, c0, c1, h1);
    };
    // three quantities over the whole row: lane s keeps x0 on lanes 0..3, x1 on 4..7,
    // x2 on 8..15
    auto tred3 = [&](double x0, double x1, double x2, int s_) __attribute__((always_inline)) {
      const bool h3 = s_ & 8, h2 = s_ & 4;
      const double a0 = tstep(kMirror{}, x0, x2, h3), a1 = tstep(kMirror{}, x1, x2, h3);
      return sstep(kXor1{}, sstep(kXor2{}, tstep(kHalfMir{}, a0, a1, h2)));
    };
    // A v on the own rows for own-column values (vf, vX), the previous stage's states in P
    auto rowA = [&](double vf, double vX, lds_cd* P, double (&ax)[3]) __attribute__((always_inline)) {
      MPCQ_LANE_OFFS(true);
      double bco[12];
#pragma unroll
      for (int psi = 0; psi < 12; ++psi) {
        const int fp = psi / 3, cp = psi % 3;
        const double v = Ab[oB0 + 24 * fp + 7 * cp];
        bco[psi] = (ph >= 9 || (isv && cp == ph - 6)) ? v : 0.0;
      }
      const double bfx = bdot_ln12(bco, vf, 0.0);
      double dyn = Ab[oXd] * vX;
      const int zP = (int)((lds_cd*)sh.zero - P);  // stage 0 has no X_0 term: read zeros, not slot -1
      const double d1 = dyn + Ab[oHd] * P[hp ? oXSp - 12 : zP];
      const double d2 = d1 + Ab[oH6] * P[hp ? oXSp6 - 12 : zP];
      dyn = hp ? (isv ? d1 : d2) : dyn;
      dyn = isv ? dyn + bfx : dyn;
      const double q0 = qbc<0>(vf), q1 = qbc<1>(vf), q2 = qbc<2>(vf);
      const double frA = Ab[oFb] * q2 + Ab[oFa] * (ta0 ? q0 : q1);
      const double frB = Ab[oF4] * q2;
      const double swg = Ab[oF + 4] * vf;
      ax[0] = cl ? dyn : frA;
      ax[1] = cl ? swg : frB;
      ax[2] = cl ? frA : 0.0;
    };
    // A' w on the own columns for own-row values w, the next stage's dynamics-row w in W
    auto colAt = [&](const double (&w)[3], const double* W, double& atf, double& atX)
        __attribute__((always_inline)) {
      MPCQ_LANE_OFFS(true);
      atf = colF_off(w);
      const double* wn = W + 12 * (k < N - 1 ? k + 1 : k);
      const double sXv = Ab[oXd] * w[0];
      const double x1 = sXv + Ab[oXd + 1] * wn[isv ? ph - 6 : ph];
      const double x2 = x1 + Ab[oXd + 2] * wn[ph];
      atX = k < N - 1 ? (isv ? x2 : x1) : sXv;
    };
    // OSQP 0.6's infeasibility tests (auxil.c is_primal_infeasible / is_dual_infeasible)
    // on the last iteration's delta_y (dy, own rows) and delta_x (dxf, dxX, own
    // columns), evaluated the way osqp evaluates them: the cheap conditions first
    // (||E dy||, u'dy+ + l'dy-, ||D dx||, ||D^-1 P dx||), the products A' dy / A dx
    // only where those hold.  infeas_cheap runs right after the update, while the
    // deltas are live: it publishes them (na / nb, free between the sweeps) with
    // update_info's states / duals under one barrier and leaves the per-wave partials
    // of the cheap quantities in red[32 wv + 16 ..]; update_info(INF) combines them
    // into uniform flags (each test only where its residual test fails, as osqp's
    // check_termination); infeas_products, only when a flag holds, adds the products
    // (two more barriers).  On MPC.py's QPs the dual side never reaches its product
    // and the primal side does at ~40 % of the checks (oracle counts, C2 batch), so
    // the product pass is skipped at most checks -- with identical outcomes.
    // outcome bits (one uniform int: the loop carries it): 1 primal, 2 dual infeasible
    // at the check's tolerances, 4 / 8 at the approximate (x10) ones
    int inf_bits = 0;
    int inf_need = 0;  // cheap-condition bits (same layout) awaiting the products
    // The termination check's scaling constants (fixed once the Ruiz scaling is done):
    // D, D^-1 of the own columns, E^-1 of the own rows, the scaled P diagonal, c and
    // 1/c.  Held across the ADMM loop, which does not use them, they were spilled and
    // each use in the check waited on its own scratch reload; they are stored once in
    // private memory instead and read back in a batch at the top of each check phase
    // (through a laundered pointer: never forwarded from the store, so nothing derived
    // from them is hoisted out of the loop either; cached scratch loads, not volatile
    // ones, which would bypass the caches).  Values and rounding are the ones the check
    // computed before (1.0 / Df etc.).
    // (the reciprocals 1 / D, 1 / E and 1 / c are divided again where the check uses them:
    // the same correctly rounded quotients, and 48 B less private memory per lane)
    enum { CK_DF, CK_DX, CK_PBF, CK_PBX, CK_C, CK_E0, CK_E1, CK_E2, CK_BND, CK_COUNT };
    double ck_mem_[CK_COUNT];
    auto ck_ptr = [&]() __attribute__((always_inline)) -> pdbl* {
      pdbl* q = (pdbl*)&ck_mem_[0];
      asm volatile("" : "+v"(q));
      return q;
    };
    // (beyond 32 stages the loop itself is short of registers: there the values are
    // derived where used, as before -- held in memory they cost the loop a spill,
    // N = 48 9.7 -> 10.4 us per iteration, profiles/r03k_iterbench.txt)
    auto ck = [&](int i) __attribute__((always_inline)) -> double {
      if constexpr (BIG) {
        switch (i) {
          case CK_DF: return Df;
          case CK_DX: return DX;
          case CK_PBF: return Pbf();
          case CK_PBX: return PbX();
          case CK_C: return cscale;
          case CK_E0: return E[0];
          case CK_E1: return E[1];
          case CK_E2: return E[2];
          default: return bnd;
        }
      } else {
        return ck_ptr()[i];
      }
    };
    // every constant of the block through one laundered pointer (one batch of loads; the
    // unused ones are dropped by the compiler)
    auto ck_all = [&](double (&cv)[CK_COUNT]) __attribute__((always_inline)) {
      if constexpr (BIG) {
#pragma unroll
        for (int i = 0; i < CK_COUNT; ++i) cv[i] = ck(i);
      } else {
        const pdbl* const q = ck_ptr();
#pragma unroll
        for (int i = 0; i < CK_COUNT; ++i) cv[i] = q[i];
      }
    };
    // The check's lane ids, re-derived from a laundered thread index: the red[] addresses
    // built from them would otherwise be hoisted out of the ADMM loop and spilled too.
#define MPCQ_CHECK_IDS()                                           \
  int tl_ = t;                                                     \
  asm volatile("" : "+v"(tl_));                                    \
  [[maybe_unused]] const int wv = tl_ >> 6, lane = tl_ & 63, s = tl_ & 15
    // The bounds as the check sees them: lo_of / hi_of from the row scaling E and the
    // dynamics bound in the check's constant block (ck, read with the others in one
    // batch).  Formed from the loop's own E / bnd, the products (-inf E, -fz_max E) were
    // hoisted out of the ADMM loop and spilled, and each came back in the check as a
    // scratch reload waited for on its own.  Same expressions, same values.
    auto chk_bounds = [&](const double (&cv)[CK_COUNT], double (&lo)[3], double (&hi)[3])
        __attribute__((always_inline)) {
      if constexpr (FUSED) {
        const double e0 = cv[CK_E0], e1 = cv[CK_E1], e2 = cv[CK_E2], bd = cv[CK_BND];
        double fz = p.fz_max;
        asm volatile("" : "+v"(fz));
        lo[0] = cl ? bd : -kInf * e0;
        lo[1] = cl ? 0.0 : -fz * e1;
        lo[2] = cl ? -kInf * e2 : -kInf;
        hi[0] = cl ? bd : 0.0;
        hi[1] = 0.0;
        hi[2] = cl ? 0.0 : kInf;
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) { lo[j] = lo_of(j); hi[j] = hi_of(j); }
      }
    };
    // the infeasibility tolerances, laundered for the same reason (10 eps, hoisted, was
    // spilled)
    auto chk_eps = [&](double& epi0, double& edi0) __attribute__((always_inline)) {
      epi0 = p.eps_prim_inf;
      edi0 = p.eps_dual_inf;
      asm volatile("" : "+v"(epi0), "+v"(edi0));
    };
    double dyp[3];     // delta_y projected onto the polar of the recession cone of [l, u]
    // The cheap part of OSQP's infeasibility tests on the last iteration's deltas, own
    // data only: dyp, and this wave's maxima ||E dy|| / ||D dx|| / ||D^-1 P dx|| and sum
    // u'dy+ + l'dy- into P[PS wv + 16 + {0, 2, 3, 6}] (red for the blocking check, dcp
    // for the deferred one).  cv: the constant block, read ahead of the check (ck_all).
    auto cheap_partials = [&](const double (&dy)[3], double dxf, double dxX, const double (&cv)[CK_COUNT],
                              double* const P, int PS) __attribute__((always_inline)) {
      MPCQ_CHECK_IDS();
      double lob[3], hib[3];
      chk_bounds(cv, lob, hib);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const bool uinf = hib[j] > kInf * kMinScaling, linf = lob[j] < -kInf * kMinScaling;
        dyp[j] = uinf ? (linf ? 0.0 : fmin(dy[j], 0.0)) : (linf ? fmax(dy[j], 0.0) : dy[j]);
      }
      double ndy = 0.0, ineq = 0.0;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double lj = lob[j], hj = hib[j];
        ndy = fmax(ndy, fabs(cv[CK_E0 + j] * dyp[j]));
        ineq += hj * fmax(dyp[j], 0.0) + lj * fmin(dyp[j], 0.0);
      }
      if (phantom) ineq = 0.0;  // a sum: stage N-1 counts once
      double q3[2] = {0.0, 0.0};
      {
        const double df = cv[CK_DF], dx = cv[CK_DX], dif = 1.0 / df, diX = 1.0 / dx;
        const double pbf = cv[CK_PBF], pbx = cv[CK_PBX];
        if (cl) {
          q3[0] = fmax(fabs(df * dxf), fabs(dx * dxX));                // ||D dx||
          q3[1] = fmax(fabs(pbf * dxf * dif), fabs(pbx * dxX * diX));  // ||D^-1 P dx||
        }
      }
      // maxima over the wave (lanes 0 / 4 / 8 keep ||E dy|| / ||D dx|| / ||D^-1 P dx||,
      // published in slots 0 / 2 / 3), the sum by xor butterflies
      const double mine = pair_max(row_pair_max(tred3(ndy, q3[0], q3[1], s)));
      ineq += dppd<0xB1>(ineq);
      ineq += dppd<0x4E>(ineq);
      ineq += dppd<0x124>(ineq);
      ineq += dppd<0x128>(ineq);
      ineq = row_pair_sum(ineq);
      {
        const long long bb = __double_as_longlong(ineq);
        const auto lo_ = __builtin_amdgcn_permlane32_swap((unsigned)bb, (unsigned)bb, false, false);
        const auto hi_ = __builtin_amdgcn_permlane32_swap((unsigned)(bb >> 32), (unsigned)(bb >> 32), false, false);
        ineq = __longlong_as_double(((long long)hi_[0] << 32) | lo_[0]) +
               __longlong_as_double(((long long)hi_[1] << 32) | lo_[1]);
      }
      if (lane == 0 || lane == 4 || lane == 8) P[PS * wv + 16 + (lane == 0 ? 0 : 2 + (lane >> 3))] = mine;
      if (lane == 6) P[PS * wv + 16 + 6] = ineq;
    };
    auto infeas_cheap = [&](const double (&dy)[3], double dxf, double dxX, const double (&cv)[CK_COUNT])
        __attribute__((always_inline)) {
      cheap_partials(dy, dxf, dxX, cv, sh.red, 32);
      // published together with update_info's states / duals, one barrier for both
      if (cl) {
        sh.u.it.na[k][ph] = dxX;
        sh.u.it.nb[k][ph] = dyp[0];
        sh.u.it.yv[k][ph] = xX;
        sh.u.it.bo[k][ph] = y[0];
      }
      sync_all();  // (update_info(INF) relies on this barrier for its own publication)
    };
    // the products, where a cheap condition holds (inf_need != 0, uniform): A' dy for
    // the primal test, A dx for the dual one, on the deltas infeas_cheap published
    // role: std::true_type (kKI's helpers) passes the barriers and forms the uniform bits only
    auto infeas_products = [&](auto role, double dxf, double dxX, const double (&cv)[CK_COUNT])
        __attribute__((always_inline)) {
      constexpr bool H = decltype(role)::value;
      MPCQ_CHECK_IDS();
      launder_p();
      if constexpr (!H) {
      double vu = -INFINITY, vl = -INFINITY;
      {
        double adx[3], lob[3], hib[3];
        rowA(dxf, dxX, (lds_cd*)&sh.u.it.na[0][0], adx);
        chk_bounds(cv, lob, hib);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const double lj = lob[j], hj = hib[j], v = adx[j] / cv[CK_E0 + j];
          if (hj < kInf * kMinScaling) vu = fmax(vu, v);
          if (lj > -kInf * kMinScaling) vl = fmax(vl, -v);
        }
      }
      double naty = 0.0;
      {
        double dtf, dtX;
        colAt(dyp, &sh.u.it.nb[0][0], dtf, dtX);
        const double dif = 1.0 / cv[CK_DF], diX = 1.0 / cv[CK_DX];
        if (cl) naty = fmax(fabs(dtf * dif), fabs(dtX * diX));  // ||D^-1 A' dy||
      }
      // lanes 0 / 4 / 8 keep ||D^-1 A' dy|| / vu / vl, published in slots 1 / 4 / 5
      const double mine = pair_max(row_pair_max(tred3(naty, vu, vl, s)));
      if (lane == 0 || lane == 4 || lane == 8) sh.red[32 * wv + 16 + (lane == 0 ? 1 : 4 + (lane >> 3))] = mine;
      }
      sync_all();
      const int e = s < 6 ? s : 0;  // slots 16..21 are all maxima (0 / 2 / 3 from infeas_cheap)
      double v = sh.red[16 + e];
#pragma unroll
      for (int w = 1; w < NW; ++w) v = fmax_hw(v, sh.red[32 * w + 16 + e]);
      const double ndy = rbc<0>(v), ndx = rbc<2>(v);  // (the cheap maxima, kept in slots 0 / 2)
      const double naty_ = rbc<1>(v), vu_ = rbc<4>(v), vl_ = rbc<5>(v);
      double epi0, edi0;
      chk_eps(epi0, edi0);
      int bits = 0;
#pragma unroll
      for (int fi = 0; fi < 2; ++fi) {
        const double f = fi == 0 ? 1.0 : 10.0, epi = f * epi0, edi = f * edi0;
        const bool pi = ((inf_need >> (2 * fi)) & 1) && naty_ < epi * ndy;
        const bool di = ((inf_need >> (2 * fi)) & 2) && !(vu_ > edi * ndx) && !(vl_ > edi * ndx);
        bits |= (pi ? 1 : 0) << (2 * fi);
        bits |= (di ? 2 : 0) << (2 * fi);
      }
      inf_bits = __builtin_amdgcn_readfirstlane(bits);
      sync_all();
    };
    // The states and dynamics-row duals are published in yv / bo, which the sweeps
    // no longer need (xs still feeds the force recovery of slower waves); lane s
    // of each row then owns residual quantity s, reduced over the wave's rows by
    // permlane swaps and over the waves through red[].  INF: also combine the
    // cheap partials of infeas_cheap into inf_need.
    // info_terms: this wave's 16 residual maxima into D[DS wv + 0..15], from the own
    // rows / columns and the published states XP (X_{k'} of stage k' at 12 (k' - 1))
    // and duals WD (y of stage k' at 12 k')
    auto info_terms = [&](const double (&cv)[CK_COUNT], lds_cd* const XP, const double* WD, double* const D,
                          int DS) __attribute__((always_inline)) {
      MPCQ_CHECK_IDS();
      const double ei3[3] = {1.0 / cv[CK_E0], 1.0 / cv[CK_E1], 1.0 / cv[CK_E2]};
      const double dif = 1.0 / cv[CK_DF], diX = 1.0 / cv[CK_DX], pbf = cv[CK_PBF], pbx = cv[CK_PBX];
      double mine, pmine;  // this lane's row maxima (tred6: primal quantity 3 b3 + (b2 ? 2 : b1))
      {  // primal side: A x - z on the own rows
        double ax[3], q6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        rowA(xf, xX, XP, ax);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const double ei = ei3[j], d = ax[j] - z[j];
          q6[0] = fmax(q6[0], fabs(ei * d));
          q6[1] = fmax(q6[1], fabs(ei * ax[j]));
          q6[2] = fmax(q6[2], fabs(ei * z[j]));
          q6[3] = fmax(q6[3], fabs(d));
          q6[4] = fmax(q6[4], fabs(ax[j]));
          q6[5] = fmax(q6[5], fabs(z[j]));
        }
        pmine = tred6(q6, s);
      }
      STAMP(5);
      {  // dual side: P x + A' y on the own columns
        double q6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        double atf, atX;
        colAt(y, WD, atf, atX);
        const double pxf = pbf * xf, pxX = pbx * xX;
        const double df_ = pxf + atf, dX_ = pxX + atX;
        if (cl) {
          q6[0] = fmax(fabs(dif * df_), fabs(diX * dX_));
          q6[1] = fmax(fabs(dif * pxf), fabs(diX * pxX));
          q6[2] = fmax(fabs(dif * atf), fabs(diX * atX));
          q6[3] = fmax(fabs(df_), fabs(dX_));
          q6[4] = fmax(fabs(pxf), fabs(pxX));
          q6[5] = fmax(fabs(atf), fabs(atX));
        }
        // the last step of the butterfly joins the sides: primal quantity e on lane
        // 2 e (e < 3) / 2 e + 2 (e >= 3), the dual's on the lane after it
        mine = tstep(kXor1{}, pmine, tred6(q6, s), s & 1);
      }
      mine = pair_max(row_pair_max(mine));  // the wave's four rows
      if (lane < 16) D[DS * wv + lane] = mine;
    };
    // info_combine: the residuals and tolerances (uniform) from every wave's partials in
    // D (stride DS); INF: the cheap infeasibility partials (slots 16..) into inf_need
    auto info_combine = [&](auto inf_tag, const double (&cv)[CK_COUNT], const double* const D, int DS)
        __attribute__((always_inline)) {
      constexpr bool INF = decltype(inf_tag)::value;
      MPCQ_CHECK_IDS();
      const double csc = cv[CK_C], cinv = 1.0 / csc;
      double qv[12];
      {
        double v = D[s];
#pragma unroll
        for (int w = 1; w < NW; ++w) v = fmax_hw(v, D[DS * w + s]);
        qv[0] = rbc<0>(v); qv[1] = rbc<2>(v); qv[2] = rbc<4>(v);
        qv[3] = rbc<8>(v); qv[4] = rbc<10>(v); qv[5] = rbc<12>(v);
        qv[6] = rbc<1>(v); qv[7] = rbc<3>(v); qv[8] = rbc<5>(v);
        qv[9] = rbc<9>(v); qv[10] = rbc<11>(v); qv[11] = rbc<13>(v);
      }
      pri_res = qv[0];
      dua_res = cinv * qv[6];
      eps_pri = p.eps_abs + p.eps_rel * fmax(qv[1], qv[2]);
      eps_dua = p.eps_abs + p.eps_rel * cinv * fmax(qv[7], qv[8]);
      s_pri = qv[3] / (fmax(qv[4], qv[5]) + kDivTol);
      s_dua = qv[9] / (fmax(qv[10], qv[11]) + kDivTol);
      // uniform by construction; readfirstlane lets the compiler see it
      pri_res = uni(pri_res); dua_res = uni(dua_res); eps_pri = uni(eps_pri);
      eps_dua = uni(eps_dua); s_pri = uni(s_pri); s_dua = uni(s_dua);

      if constexpr (INF) {
        // the cheap conditions of infeas_cheap: slots 0 ||E dy||, 2 ||D dx||, 3 ||D^-1 P dx||, 6 u'dy+ + l'dy-
        const int e = s == 2 || s == 3 || s == 6 ? s : 0;
        double v = D[16 + e];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
          const double t2 = D[DS * w + 16 + e];
          v = s == 6 ? v + t2 : fmax_hw(v, t2);
        }
        // kept in VGPRs (every lane holds the same values) and folded into one uniform
        // int at the end: SGPRs here would push loop-carried scalars into VGPR lanes
        // (v_readlane on the hot path, measured)
        const double ndy = rbc<0>(v), ndx = rbc<2>(v), npdx = rbc<3>(v), ineq = rbc<6>(v);
        double epi0, edi0;
        chk_eps(epi0, edi0);
        int need = 0;
#pragma unroll
        for (int fi = 0; fi < 2; ++fi) {
          const double f = fi == 0 ? 1.0 : 10.0, epi = f * epi0, edi = f * edi0;
          const bool pi = !(pri_res < f * eps_pri) && ndy > kDivTol && ineq < epi * ndy;
          const bool di = !(dua_res < f * eps_dua) && ndx > kDivTol && 0.0 < csc * edi * ndx &&
                          npdx < csc * edi * ndx;
          need |= (pi ? 1 : 0) << (2 * fi);
          need |= (di ? 2 : 0) << (2 * fi);
        }
        inf_need = __builtin_amdgcn_readfirstlane(need);
        inf_bits = 0;
      }
    };
    // INF: after infeas_cheap, which has published the states / duals with its deltas
    auto update_info = [&](auto inf_tag, const double (&cv)[CK_COUNT]) __attribute__((always_inline)) {
      constexpr bool INF = decltype(inf_tag)::value;
      if constexpr (!INF) {
        if (cl) { sh.u.it.yv[k][ph] = xX; sh.u.it.bo[k][ph] = y[0]; }
        sync_all();
      }
      STAMP(4);
      launder_p();
      info_terms(cv, (lds_cd*)&sh.u.it.yv[0][0], &sh.u.it.bo[0][0], sh.red, 32);
      sync_all();
      STAMP(8);
      info_combine(inf_tag, cv, sh.red, 32);
      sync_all();
    };
    auto converged = [&](double fac) __attribute__((always_inline)) {
      return pri_res < fac * eps_pri && dua_res < fac * eps_dua;
    };

    if (status == 0) {
      STAMP(0);
      // ------------------------------------------------------------ Ruiz scaling
      {
        double Pf = P0f, PX = P0X;
        double* Ex = gh0;  // row factors of this pass: Ex[48 k + 3 s + slot]
        // friction row t of foot fp: owner lane / slot
        auto fr_E = [&](int kk, int fp, int t_) __attribute__((always_inline)) {
          return t_ < 3 ? Ex[48 * kk + 3 * (4 * fp + t_) + 2] : Ex[48 * kk + 3 * (4 * fp + 3) + (t_ - 3)];
        };
        auto dyn_E = [&](int kk, int i) __attribute__((always_inline)) { return Ex[48 * kk + 3 * LN(i)]; };
        auto fr_norm = [&](int t_) __attribute__((always_inline)) {
          double v = fabs(Ab[FO<N>(k, f, 2) + 5 + t_]);
          if (t_ < 4) v = fmax(v, fabs(Ab[FO<N>(k, f, t_ >> 1) + 5 + (t_ & 1)]));
          return v;
        };
        for (int it = 0; it < p.scaling; ++it) {
          double dtf = fabs(Pf);
          {
            const int cnt = cc < 2 ? 7 : 10;
            for (int e = 0; e < cnt; ++e) dtf = fmax(dtf, fabs(Ab[fo + e]));
          }
          double dtx = fabs(PX);
          {
            const int cnt = (k < N - 1) ? (ph < 6 ? 2 : 3) : 1;
            for (int h = 0; h < cnt; ++h) dtx = fmax(dtx, fabs(Ab[xo + h]));
          }
          double et[3];
          {
            double v = fabs(Xd(k, ph));
            if (k >= 1) {
              v = fmax(v, fabs(Hd(k, ph)));
              if (ph < 6) v = fmax(v, fabs(H6(k, ph)));
            }
            if (ph >= 6) {
#pragma unroll
              for (int psi = 0; psi < 12; ++psi) v = fmax(v, fabs(Bc(k, ph, psi / 3, psi % 3)));
            }
            et[0] = cl ? v : fr_norm(3);
            et[1] = cl ? fabs(Ab[fo + 4]) : fr_norm(4);
            et[2] = cl ? fr_norm(c) : 0.0;
          }
          dtf = dtf < kMinScaling ? 1.0 : (dtf > kMaxScaling ? kMaxScaling : dtf);
          dtx = dtx < kMinScaling ? 1.0 : (dtx > kMaxScaling ? kMaxScaling : dtx);
          dtf = 1.0 / sqrt(dtf);
          dtx = 1.0 / sqrt(dtx);
          Df *= dtf;
          DX *= dtx;
          Pf = dtf * Pf * dtf;
          PX = dtx * PX * dtx;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            double v = et[j];
            v = v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v);
            et[j] = 1.0 / sqrt(v);
            E[j] *= et[j];
          }
#pragma unroll
          for (int j = 0; j < 3; ++j) Ex[48 * k + 3 * s + j] = et[j];
          sync_all();
          if (cl && !phantom) {  // own columns: E_row A D_col (in place: phantom rows keep out)
            const double dA = dyn_E(k, 6 + cc);
            AbW[fo] = dA * AbW[fo] * dtf;
#pragma unroll
            for (int j = 0; j < 3; ++j) AbW[fo + 1 + j] = dyn_E(k, 9 + j) * AbW[fo + 1 + j] * dtf;
            AbW[fo + 4] = et[1] * AbW[fo + 4] * dtf;
            if (cc < 2) {
              AbW[fo + 5] = fr_E(k, f, 2 * cc) * AbW[fo + 5] * dtf;
              AbW[fo + 6] = fr_E(k, f, 2 * cc + 1) * AbW[fo + 6] * dtf;
            } else {
#pragma unroll
              for (int t_ = 0; t_ < 5; ++t_) AbW[fo + 5 + t_] = fr_E(k, f, t_) * AbW[fo + 5 + t_] * dtf;
            }
            AbW[xo] = et[0] * AbW[xo] * dtx;
            if (k < N - 1) {
              if (ph >= 6) {
                AbW[xo + 1] = dyn_E(k + 1, ph - 6) * AbW[xo + 1] * dtx;
                AbW[xo + 2] = dyn_E(k + 1, ph) * AbW[xo + 2] * dtx;
              } else {
                AbW[xo + 1] = dyn_E(k + 1, ph) * AbW[xo + 1] * dtx;
              }
            }
          }
          // cost scaling: c = 1 / max(mean |P|, 1)  (q = 0)
          double ps = cl && !phantom ? fabs(Pf) + fabs(PX) : 0.0;
          ps = wave_sum(ps);
          if ((t & 63) == 0) sh.red[wv] = ps;
          sync_all();
          ps = 0.0;
#pragma unroll
          for (int w = 0; w < NW; ++w) ps += sh.red[w];
          const double mean = ps / n;
          double ctmp = mean > 1.0 ? mean : 1.0;
          ctmp = ctmp < kMinScaling ? 1.0 : (ctmp > kMaxScaling ? kMaxScaling : ctmp);
          ctmp = 1.0 / ctmp;
          Pf *= ctmp;
          PX *= ctmp;
          cscale = uni(cscale * ctmp);
          sync_all();
        }
      }
      // scaled bounds, constraint classes (osqp set_rho_vec)
      if constexpr (FUSED) {
        bnd *= E[0];
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) { lo_g[j] *= E[j]; hi_g[j] *= E[j]; }
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double lj = lo_of(j), hj = hi_of(j);
        unsigned cj;
        if (lj < -kInf * kMinScaling && hj > kInf * kMinScaling) cj = RC_LOOSE;
        else if (hj - lj < kRhoTol) cj = RC_EQ;
        else cj = RC_INEQ;
        cls |= cj << (2 * j);
      }
      set_rho();
      zc_store();
      if constexpr (!BIG) {
        pdbl* const q = ck_ptr();
        q[CK_DF] = Df; q[CK_DX] = DX; q[CK_PBF] = Pbf(); q[CK_PBX] = PbX(); q[CK_C] = cscale;
        q[CK_E0] = E[0]; q[CK_E1] = E[1]; q[CK_E2] = E[2]; q[CK_BND] = bnd;
      }
      // warm start (osqp_warm_start: x = D^-1 x0, z = A x; y = c E^-1 y0)
      if (a.warm_x) {
        xf = a.warm_x[b * n + colF] / Df;
        xX = a.warm_x[b * n + colX] / DX;
        if (cl) sh.u.it.xs[k + 1][ph] = xX;
        sync_all();
        row_A(xf, xX, z);
        if (!cl) z[2] = 0.0;
        sync_all();
      }
      if (a.warm_y) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int r = nat_row(j);
          // dual_warm = 1: osqp's workspace y from the previous solve, kept as is across the
          // re-scaled update(Ax=) (MPC.py:419-420); 0: osqp_warm_start_y's scaling
          const double wy = r >= 0 ? a.warm_y[b * m + r] : 0.0;
          y[j] = r >= 0 ? (p.dual_warm ? wy : cscale * wy / E[j]) : 0.0;
        }
      }
      // a resumed slice (mpcq_set_slice): the iterate every lane held when it was suspended
      if constexpr (kSlice<N> && !KI) {
        if (a.resume) {
          constexpr int64_t RL = res_lanes(N);
          const double* const q = a.res + b * 8 * RL + t;
          xf = q[0];
          xX = q[RL];
#pragma unroll
          for (int j = 0; j < 3; ++j) { z[j] = q[(2 + j) * RL]; y[j] = q[(5 + j) * RL]; }
        }
      }
      sync_all();
      STAMP(1);

      // The phases of one KKT solve (K w = b, K = P + sigma I + A'RA as factored):
      // ph_rhs publishes the sweep right-hand sides of b = xc + A' w (P1-P4), ph_sweep
      // runs the state sweeps (P5-P7), ph_recover the forces and A w on the own rows
      // (P8, P9's first half).  The ADMM loop calls them with admm = true (w = rho z - y,
      // xc = sigma x); polish with its own w and x terms.
      // the iteration-invariant LDS operands of ph_rhs (A_f column, F W column, the
      // state column's dynamics coefficients)
      // (kColfFold, round 5) A_f's first coefficient masked by the force component: cf0m[j] =
      // cf[0] on the lanes of component j (2: every other), else 0, so the component-dependent
      // row broadcast of colF folds into v_fmac_f64_dpp.  With the right-hand-side phase's
      // pointer laundering dropped (below) the phase lost ~40 instructions per wave and
      // iteration: same box (profiles/r05p_*, r05q_*), N = 16 1.851-1.872 -> 1.788-1.791 us
      // per iteration alone, 2.18-2.21 -> 2.134-2.142 at two per CU, N = 32 3.105-3.124 ->
      // 2.966-2.982; C2 125.3 k -> 130.7 k QP/s.  The same terms in the same order (the
      // compiler's own contraction of colF had rounded A_2 w_10 first, so the last bits of
      // b_f differ from round 4's); statuses and iterations equal to the oracle's.  Up to 32
      // stages: beyond, that last-bit change moved the N = 48 session loop's fifth tick
      // 1.01e-7 from the oracle (its test allows 1e-7; r05r), and the loop reads its operands
      // per iteration there anyway.  Dropping the checks' laundering as well was slower at
      // N = 32 (3.06 us, r05q).
      constexpr bool kColfFold = !KI && !BIG;
      struct RhsOps {
        double cf[10], fwc[12], cXd, cHd, cH6;
        double cf0m[kColfFold ? 3 : 1];
      };
      auto load_rhs_ops = [&](RhsOps& o) __attribute__((always_inline)) {
        MPCQ_LANE_OFFS(true);  // (once per stretch of iterations)
#pragma unroll
        for (int i = 0; i < 10; ++i) o.cf[i] = Ab[oF + i];
        if constexpr (kColfFold) {
          const int cs = cc == 0 ? 0 : (cc == 1 ? 1 : 2);
#pragma unroll
          for (int j = 0; j < 3; ++j) o.cf0m[j] = cs == j ? o.cf[0] : 0.0;
        }
#pragma unroll
        for (int psi = 0; psi < 12; ++psi) o.fwc[psi] = FWr[oFWcm + 6 * psi];
        o.cXd = Ab[oXd];
        o.cHd = Ab[oHdm];
        o.cH6 = Ab[oH6m];
      };
      // o: the operands held in registers (the ADMM loop), or null: read them here (polish,
      // whose loop would otherwise spill them)
      // rsum (kKI): r = bo + na summed in LDS (two ds_add_f64 into a zeroed slot: its two
      // addends commute, so the sum's bits do not depend on which lane adds first) instead of
      // bo / na stored apart -- the product then loads one value per column, not two and an add
      auto ph_rhs = [&](bool admm, const RhsOps* op, const double (&pw)[3], double xcf, double xcX, double& uf,
                        double& beta, lds_d* rsum = nullptr) __attribute__((always_inline)) {
          // (up to 48 stages no launder_p here since round 5: the laundered base pointers
          // cost ~40 instructions per iteration and the loop has no spill without them; beyond
          // 48 stages, at 128 VGPRs, the iteration was 15.0 -> 16.9 us without, r05r)
          if constexpr (kFrWork<N>) launder_p();
          RhsOps own_;
          if (!op) load_rhs_ops(own_);
          const RhsOps& o = op ? *op : own_;
          MPCQ_LANE_OFFS(kRecompLoop);
          // beyond 48 stages (kFrWork) the F_k row is read from the workspace here (issued first,
          // its latency behind the phase's other loads) instead of being held through
          // the ADMM loop in 24 of the 128 VGPRs
          double frg[12];
          if constexpr (kFrWork<N>) {
            g_cd* q = FRg;
            asm volatile("" : "+v"(q));
#pragma unroll
            for (int i = 0; i < 12; ++i) frg[i] = q[16 * NR * i];
          }
          // P1-P4: w = rho z - y; b_f = sigma x_f + A_f' w and u = F b_f, beta = R B u
          // (stage-local, DPP only); then the sweep right-hand side of the own state
          // column (bo) and this stage's dynamics-row terms of stage k-1's state
          // columns (na, nb): the only LDS hand-off before the sweeps.
          // every LDS operand of this phase is iteration-invariant: issue all the loads
          // first (one LDS round trip instead of one per use)
          const double cXd = o.cXd, cHd = o.cHd, cH6 = o.cH6;
          double w[3];
#pragma unroll
          for (int j = 0; j < 3; ++j) w[j] = admm ? rr[j] * z[j] - y[j] : pw[j];
          if constexpr (kZcMem<N>) {
            if (admm) {
              pdbl* const q = zc_ptr();
              const double r0 = q[ZC_RR], r1 = q[ZC_RR + 1], r2 = q[ZC_RR + 2];
              w[0] = r0 * z[0] - y[0];
              w[1] = r1 * z[1] - y[1];
              w[2] = r2 * z[2] - y[2];
            }
          }
          // the phase's arithmetic starts after this point, the loads before it
          asm volatile("" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]) : : "memory");
          double colf;
          if constexpr (kColfFold) {
            // colF_c's six row-broadcast terms folded into v_fmac_f64_dpp (the masked terms
            // add exact zeros); the quad-broadcast terms as there
            double sA = -0.0, sB = -0.0;
            asm("s_nop 1\n\t"
                "v_fmac_f64_dpp %0, %2, %3 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %1, %2, %4 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %0, %2, %5 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %1, %2, %6 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %0, %2, %7 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %0, %2, %8 row_newbcast:13 row_mask:0xf bank_mask:0xf"
                : "+v"(sA), "+v"(sB)
                : "v"(w[0]), "v"(o.cf0m[0]), "v"(o.cf[1]), "v"(o.cf0m[1]), "v"(o.cf[3]), "v"(o.cf0m[2]),
                  "v"(o.cf[2]));
            static_assert(LN(6) == 8 && LN(7) == 9 && LN(8) == 10 && LN(9) == 12 && LN(10) == 13 && LN(11) == 14,
                          "the broadcast lanes above");
            const double wf0 = qbc<0>(w[2]), wf1 = qbc<1>(w[2]), wf2 = qbc<2>(w[2]);
            const double wf3 = qbc<3>(w[0]), wf4 = qbc<3>(w[1]);
            const double* const A = o.cf;
            sA += A[4] * w[1];
            sB += A[5] * (cc == 1 ? wf2 : wf0);
            sA += A[6] * (cc == 1 ? wf3 : wf1);
            const double sC = (A[7] * wf2 + A[8] * wf3) + A[9] * wf4;
            colf = (sA + sB) + m2 * sC;
          } else {
            colf = colF_c(o.cf, w);
          }
          const double bf = colf + (admm ? p.sigma * xf : xcf);  // b_f = sigma x_f + A_f' w (- q, q = 0)
          // u = F b_f (kept for the forces) and beta = R B u = (F W)' b_f (rows 6..11)
          if constexpr (kFrWork<N>) {
            uf = bdot_ln12(frg, bf, 0.0);
          } else {
            uf = bdot_ln12(Fr, bf, 0.0);
          }
          beta = bdot_ln12(o.fwc, bf, 0.0);
          {
            const double wd = w[0] - beta;  // dynamics-row w less the force Schur term (beta = 0 on rows 0..5)
            const double bo = (admm ? p.sigma * xX : xcX) + cXd * wd;
            const double na = cHd * wd;                  // Hd(k, ph): on X_k[ph], stage k-1's column ph
            const double nb = cH6 * w[0];                // H6(k, ph): on X_k[ph+6] (ph < 6)
            // stage 0 zeroes the last stage's na / nb (that stage has no next stage:
            // its coefficients read zero)
            if (!(KI && rsum)) *(cl ? Wbo : Wdump) = bo;
            // stage k-1's component r takes na of lane r and nb of the lane 8 away in the
            // row (component r -+ 6, LN): summed here, one value and one add less per
            // sweep step
            const double nbx = dppd<0x128>(nb);  // row_ror:8
            if (KI && rsum) {
              if (cl) {
                __hip_atomic_fetch_add(rsum + 12 * k + ph, bo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(rsum + 12 * (k >= 1 ? k - 1 : N - 1) + ph, na + nbx, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
              }
            } else {
              *(cl ? Wna : Wdump) = na + nbx;
            }
            if constexpr (kND<N>) {  // B's phantom reads a zero right-hand side (the checks scribble on u.it)
              if (k == NDS<N> && cl) {
                sh.u.it.bo[kPhRhs<N>][ph] = 0.0;
                sh.u.it.na[kPhRhs<N>][ph] = 0.0;
              }
            }
          }
          // (the barrier that publishes bo / na / nb opens ph_sweep)
      };
      auto ph_sweep_split = [&]() __attribute__((always_inline)) {
          // P5-P7: the state solve.  The two chains run on wave 0, each on a pair of rows
          // that splits every 12-term row product in two: rows 0 / 1 (top / bottom chain)
          // take the first six terms and the right-hand side, rows 2 / 3 the last six, and
          // one permlane32 swap-add joins the halves (rows 0 + 2, 1 + 3).  Rows 2 / 3 hold
          // the chain vector rotated by six lanes (row_ror:10), so both halves broadcast
          // from lanes 0..5 with the same instruction.  Inward step j = 1..MID: y_kk =
          // b_kk - G_kk y_kk(j-1) (top kk = j, G_kk in GH slot j; bottom kk = N-1-j, H_kk
          // in slot MID+j, stopping after BOT steps), each y stored to its stage's yv slot;
          // step MID+1: the meeting stage x_m = M^{-1} (y_m + v_m - b_m) (the two pairs
          // joined by permlane16).  Then, on every wave, w_k = S_k^{-1} y_k stage-parallel
          // (one barrier pair); then the outward steps x_kk = w_kk - G' x_next on wave 0.
          // Used beyond 32 stages, where S^{-1} lives in L2 (N = 48: 13.9 -> 12.9 us per
          // iteration); up to 32 stages ph_sweep_lag is faster (N = 16: 1.90 vs 2.31 us,
          // N = 32: 3.31 vs 3.92, profiles/r03h_iterbench.txt): the split saves six FMAs and
          // three row reads per step but adds the swap-add, the rotation and the selects,
          // and the stage-parallel S^{-1} phase with its two barriers.
          int tl_ = t;  // (laundered: the lane ids derived here are not hoisted out of the loop and spilled)
          asm volatile("" : "+v"(tl_));
          const int hi = (tl_ >> 5) & 1;  // rows 2 / 3: the second six terms
          const int h6 = 6 * hi;
#ifndef MPCQ_REP_SWEEP
#define MPCQ_REP_SWEEP 1
#endif
#pragma nounroll
          for (int rep_ = 0; rep_ < MPCQ_REP_SWEEP; ++rep_) {  // > 1: timing experiments only
          double xp = 0.0;
          double g[6];
          // lane rr of a row reads entries h6..h6+5 of row rr of the step's matrix
          // (16-B aligned: 3 ds_read_b128); the bottom chain's slots sit past N/2 (+2, SLOT)
          lds_cd* const Mb = GHr + (GS * (cr == 0 ? 0 : MID) + (cr == 0 ? 0 : kSlotPad<N>) + RS * rr_ + h6);
          auto row6 = [&](lds_cd* q) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              const dbl2 v = ((lds_cd2*)q)[i];
              g[2 * i] = v.x;
              g[2 * i + 1] = v.y;
            }
          };
          // step j's rows (j a constant after unrolling); the bottom chain's steps past BOT
          // (even N) re-read its last matrix, their products discarded by the hand-off select
          auto rowp = [&](int j) __attribute__((always_inline)) -> lds_cd* {
            if (j <= BOT) return Mb + GS * j;
            return Mb + GS * (cr == 0 ? j : BOT);
          };
          STAMP(15);  // (diagnostic builds: the own right-hand side, then the wait for the others)
          if (t < 64) row6(rowp(1));
          sync_all();
          STAMP(3);
          // outward step j reads G_{MID-j+1}' (top, slot MID+1-j) / H_{MID+j-1}' (bottom,
          // slot N-j): column rr, entries h6..h6+5 (LDS offsets are unsigned, so the bases
          // sit at the lowest slot a chain reaches)
          lds_cd* const Ob = GHr + (GS * (cr == 0 ? 1 : N - MID) + (cr == 0 ? 0 : kSlotPad<N>) + rr_ + RS * h6);
          // (kLagOut) the same columns read whole: lane rr takes all 12 entries of column rr
          [[maybe_unused]] lds_cd* const ObL = GHr + (GS * (cr == 0 ? 1 : N - MID) + (cr == 0 ? 0 : kSlotPad<N>) + rr_);
          [[maybe_unused]] double go[kLagOut<N> ? 12 : 1];
          if (t < 64) {
            // the sweeps are every wave's critical path (the other waves of the instance
            // wait at the barrier): issue them ahead of a co-resident instance's phases
            __builtin_amdgcn_s_setprio(3);
            // right-hand side of step j (rows 0 / 1 add it): top stage j (slot j), bottom
            // stage N-1-j (slot MID+1+j; the meeting stage MID at the bottom's step BOT,
            // slot MID, which the bottom re-reads in the steps it does not take); na at +12N
            lds_cd* const Bb = (lds_cd*)&sh.u.it.bo[0][0] + (12 * (cr == 0 ? 0 : MID + 1) + rr_);
            lds_cd* const Bm = (lds_cd*)&sh.u.it.bo[MID][rr_];
            auto rhs = [&](int j) __attribute__((always_inline)) -> lds_cd* {  // j: a constant
              return (j >= BOT && cr != 0) ? Bm : Bb + 12 * j;
            };
            // the index a lane holds in the broadcast layout (rows 2 / 3: rotated by six)
            const int ri = hi ? (rr_ < 6 ? rr_ + 6 : rr_ - 6) : rr_;
            lds_d* const sink = (lds_d*)&sh.red[0] + (t & 31);
            // y of step j's stage from rows 0 / 1 (top slot j, bottom slot MID+1+j: SIG)
            lds_d* const Yh = (hi == 0 && s < 12) ? (lds_d*)&sh.u.it.yv[0][0] + (12 * (cr == 0 ? 0 : MID + 1) + rr_)
                                                  : sink;
            // y_kk(0) = b of the chain's first stage, in the broadcast layout; the next two
            // right-hand sides in the output layout (published by the barrier just passed:
            // loaded together, waited for once)
            lds_cd* const B0 = (lds_cd*)&sh.u.it.bo[0][0] + (12 * (cr == 0 ? 0 : MID + 1) + ri);
            double s0 = B0[0], s1 = B0[12 * N];
            double c0 = rhs(1)[0], c1 = rhs(1)[12 * N];
            asm volatile("" : "+v"(s0), "+v"(s1), "+v"(c0), "+v"(c1));
            double src = s0 + s1;
            *Yh = src;  // (rows 0 / 1: the broadcast layout is the output layout)
            double bcn = hi ? 0.0 : c0 + c1;
            double b0 = rhs(2)[0], b1 = rhs(2)[12 * N];
#pragma unroll
            for (int j = 1; j <= MID + 1; ++j) {
              asm volatile("" : : : "memory");
              double gc[6];
#pragma unroll
              for (int i = 0; i < 6; ++i) gc[i] = g[i];
              const double bc = j <= MID ? bcn : 0.0;
              if (j < MID) {  // prefetch the next step's rows
                row6(rowp(j + 1));
              } else if (j == MID) {  // the meeting step: M^{-1} (slot 0) and b_m in the broadcast layout
                row6(GHr + RS * rr_ + h6);
                lds_cd* qb = (lds_cd*)&sh.u.it.bo[MID][ri];
                b0 = qb[0]; b1 = qb[12 * N];
              } else if constexpr (kLagOut<N>) {  // the last step: the first outward step's columns (12 terms)
#pragma unroll
                for (int i = 0; i < 12; ++i) go[i] = ObL[RS * i + GS * (MID - 1)];
              } else {  // the last step: the first outward step's columns
#pragma unroll
                for (int i = 0; i < 6; ++i) g[i] = Ob[RS * i + GS * (MID - 1)];
              }
              asm volatile("" : : : "memory");  // the prefetch is issued here, not sunk to its use
              double s_in = src;
              if (j == MID + 1) s_in = row_pair_sum(src) - (b0 + b1);
              const double y = pair_sum32(bdot6(gc, s_in, bc));
              // the next right-hand side is summed after the chain: its loads were issued at
              // the end of the previous step, and summing them ahead of the chain would put
              // their LDS latency on the critical path
              asm volatile("" : "+v"(b0), "+v"(b1));
              if (j < MID) bcn = hi ? 0.0 : b0 + b1;
              if (j + 2 <= MID) {
                b0 = rhs(j + 2)[0]; b1 = rhs(j + 2)[12 * N];
              }
              // row_ror:10 (lane q <- lane q + 6) on every lane, then a select: as a select on
              // the rotated value the compiler kept an exec-masked branch, and the register
              // copies in front of it waited for the right-hand-side loads just issued (an LDS
              // round trip per step)
              double yr = dppd<0x12A>(y);
              asm volatile("" : "+v"(yr));
              const double yb = hi ? yr : y;
              if (j <= MID) {
                // y of stage kk(j) (the meeting stage's y_m / v_m stay in registers); the
                // bottom chain keeps its v_m through the steps past BOT
                if (j < MID) *((cr == 0 || j < BOT) ? Yh + 12 * j : sink) = y;
                const bool adv = j <= BOT || cr == 0;
                src = adv ? yb : src;
              } else {
                // (kLagOut: the outward products are full rows on every row pair, so every
                // row takes x_m in its own layout; pair_sum32 left it bit-identical in rows
                // 0 / 2 and 1 / 3)
                xp = kLagOut<N> ? y : yb;
                if (cr == 0 && hi == 0 && s < 12) sh.u.it.xs[SIGX<N>(MID + 1)][rr_] = y;
              }
            }
            STAMP(6);
          }
          {
            // w_k = S_k^{-1} y_k for every stage but the meeting one, stage-parallel: lane
            // LN(ph) of stage k's row takes row ph of S_k^{-1} and y_k by row broadcast
            sync_all();
            using scd2 = std::conditional_t<BIG, const dbl2, lds_cd2>;
            const scd2* const q = (scd2*)(SmR + SLOT<N>(SIG<N>(k)) + RS * ph);
            double srow[12];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              const dbl2 v = q[i];
              srow[2 * i] = v.x;
              srow[2 * i + 1] = v.y;
            }
            // (the meeting stage has no y / w: its lanes read stage 0's y, their product unused)
            double* const yk = &sh.u.it.yv[SIG<N>(k == MID ? 0 : k)][ph];
            const double wk = bdot_ln12(srow, *yk, 0.0);
            // in place: the row's reads of y_k precede (DPP operands); phantom rows keep out
            // (stage N-1's row may sit in another wave and read y after their store)
            if (cl && k != MID && !phantom) *yk = wk;
            sync_all();
          }
          if (t < 64) {
            // Outward step j: top kk = MID-j: X_kk = w_kk - G_{kk+1}' X_{kk+1}; bottom
            // kk = MID+j: X_kk = w_kk - H_{kk-1}' X_{kk-1}.  w of stage kk: top slot MID-j,
            // bottom slot N-j (Wb - 12 j); X_kk = xs[kk+1]: top slot MID+1-j, bottom slot
            // N-j (SIGX; Xb - 12 j).  Even N: the bottom chain has no step MID (its store
            // goes to the sink).  (bases at step MID's slot: step j at base + 12 (MID - j))
            lds_cd* const Wb = (lds_cd*)&sh.u.it.yv[0][0] + (12 * (cr == 0 ? 0 : N - MID) + rr_);
            lds_d* const sinkO = (lds_d*)&sh.red[0] + (t & 31);
            lds_d* const Xb = (hi == 0 && s < 12) ? (lds_d*)&sh.u.it.xs[0][0] + (12 * (cr == 0 ? 1 : N - MID) + rr_)
                                                  : sinkO;
            double bq = Wb[12 * (MID - 1)];
            if constexpr (kLagOut<N>) {
              // full 12-term column products on every row (rows 2 / 3 repeat rows 0 / 1): one
              // v_fmac chain per step, no swap-add, rotation or select (as ph_sweep_lag)
#pragma unroll
              for (int j = 1; j <= MID; ++j) {
                asm volatile("" : : : "memory");
                double gc[12];
#pragma unroll
                for (int i = 0; i < 12; ++i) gc[i] = go[i];
                const double bc = bq;
                if (j < MID) {
#pragma unroll
                  for (int i = 0; i < 12; ++i) go[i] = ObL[RS * i + GS * (MID - j - 1)];
                  if (j + 1 <= BOT) bq = Wb[12 * (MID - j - 1)];
                  else bq = Wb[12 * (MID - (cr == 0 ? j + 1 : BOT))];
                }
                asm volatile("" : : : "memory");
                const double acc = bdot12(gc, xp, bc);  // x = w - G' x_next with -G stored
                if (j < MID) {
                  xp = acc;
                  Xb[12 * (MID - j)] = acc;
                } else if constexpr (N & 1) {
                  *Xb = acc;
                } else {
                  *(cr == 0 ? Xb : sinkO) = acc;
                }
              }
            } else {
#pragma unroll
            for (int j = 1; j <= MID; ++j) {
              asm volatile("" : : : "memory");
              double gc[6];
#pragma unroll
              for (int i = 0; i < 6; ++i) gc[i] = g[i];
              const double bc = hi ? 0.0 : bq;
              if (j < MID) {
#pragma unroll
                for (int i = 0; i < 6; ++i) g[i] = Ob[RS * i + GS * (MID - j - 1)];
                // (even N: the bottom chain has no step MID; it re-reads its last w)
                if (j + 1 <= BOT) bq = Wb[12 * (MID - j - 1)];
                else bq = Wb[12 * (MID - (cr == 0 ? j + 1 : BOT))];
              }
              asm volatile("" : : : "memory");
              const double x = pair_sum32(bdot6(gc, xp, bc));  // x = w - G' x_next with -G stored
              if (j < MID) {
                double xr = dppd<0x12A>(x);
                asm volatile("" : "+v"(xr));
                xp = hi ? xr : x;
                Xb[12 * (MID - j)] = x;
              } else if constexpr (N & 1) {
                *Xb = x;
              } else {  // even N: the bottom chain has no step MID
                *(cr == 0 ? Xb : sinkO) = x;
              }
            }
            }
            __builtin_amdgcn_s_setprio(0);
          }
          wave_sync();
          }  // MPCQ_REP_SWEEP
      };
      // ph_recover's iteration-invariant operands (F W and R^{-1} Q rows, friction coefficients)
      struct RecPre {
        double fwl[6], qll[6], cFb, cFa, cF4;
      };
      auto rec_pre = [&](RecPre& r) __attribute__((always_inline)) {
        MPCQ_LANE_OFFS(kRecompLoop);
#pragma unroll
        for (int i = 0; i < 3; ++i) {  // 16-B aligned pairs: ds_read_b128 (twice ds_read2_b64's LDS rate)
          using wcd2 = std::conditional_t<BIG, const dbl2, lds_cd2>;
          const dbl2 fa = ((lds_cd2*)(FWr + oFW))[i], qa = ((wcd2*)(QLr + oQLm))[i];
          r.fwl[2 * i] = fa.x; r.fwl[2 * i + 1] = fa.y;
          r.qll[2 * i] = qa.x; r.qll[2 * i + 1] = qa.y;
        }
        r.cFb = Ab[oFb]; r.cFa = Ab[oFa]; r.cF4 = Ab[oF4];
      };
      // (kND) The state solve by nested dissection: the halves swept at once (A on wave 0, B on
      // wave 1, each ph_sweep_lag's two-ended sweep on its own slots); wave 0 then forms
      // P z_{S-1} and wave 1 Q z_{S+1} (each on its sweep lanes, lane r = component r: the half's
      // separator-side state and the P / Q rows from LDS), the separator row's lanes Sigma^{-1}
      // b_S meanwhile (b_S is published); one barrier; then every lane sums the separator's
      // states x_S = Sigma^{-1} b_S + P z_{S-1} + Q z_{S+1} and corrects its own:
      // x_k = z_k - W_k x_S.  ph_recover's barrier publishes the corrected states.  pre: the
      // iteration-invariant operands of ph_recover, read right after the sweeps (their latency
      // -- L2 for the constraint values -- behind the barrier and the correction).
      auto ph_sweep_nd = [&](RecPre* pre) __attribute__((always_inline)) {
        if constexpr (kND<N>) {
          constexpr int S = NDS<N>;
          const int wq = __builtin_amdgcn_readfirstlane(t >> 6);
          lds_d* const part = (lds_d*)&sh.nd.Part[0][0];  // [0]: P z_{S-1}, [1]: Q z_{S+1}, [2]: Sigma^{-1} b_S
          nd_sweep_halves();
          STAMP(7);  // (diagnostic builds, kND: bucket 7 the outward sweep, 4 the separator terms, 5 the
                     // barrier after them, 8 the correction; ph_recover's own wait joins bucket 7)
          if (wq < 2) {  // (the sweep's own wave_sync has published its states to the wave)
            // (lane ids from a laundered thread index: held across the loop, these addresses were
            // spilled and each reload waited for)
            int tl_ = t;
            asm volatile("" : "+v"(tl_));
            const int ri = (tl_ & 15) < 12 ? (tl_ & 15) : (tl_ & 15) - 12;
            const double zv = sh.u.it.xs[XSL<N>(wq == 0 ? S - 1 : S + 1)][ri];
            double pr[12];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              const dbl2 v = ((lds_cd2*)&sh.nd.Sep[1 + wq][RS * ri])[i];
              pr[2 * i] = v.x; pr[2 * i + 1] = v.y;
            }
            const double pz = bdot12(pr, zv, 0.0);
            if (((tl_ >> 4) & 3) == 0 && (tl_ & 15) < 12) part[12 * wq + ri] = pz;
          } else if (k == S) {
            double Si[12];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              const dbl2 v = ((lds_cd2*)&sh.nd.Sep[0][RS * ph])[i];
              Si[2 * i] = v.x; Si[2 * i + 1] = v.y;
            }
            const double bs = sh.u.it.bo[RSL<N>(S)][ph] + sh.u.it.na[RSL<N>(S)][ph];  // b_S
            const double sb = bdot_ln12(Si, bs, 0.0);
            if (cl) part[24 + ph] = sb;
          }
          if (pre) rec_pre(*pre);
          // this stage's spike row, read before the barrier (the waves that did not sweep have
          // them in registers when it opens; after it, every wave's reads met in the LDS at once)
          double Wr[12];
#pragma unroll
          for (int i = 0; i < 6; ++i) {
            const dbl2 v = ((lds_cd2*)&sh.nd.Wsp[WSI<N>(k == NDS<N> ? k - 1 : k)][RS * ph])[i];  // (the separator's product is unused)
            Wr[2 * i] = v.x; Wr[2 * i + 1] = v.y;
          }
          STAMP(4);
          sync_all();  // z of both halves, the separator's three terms
          STAMP(5);
          const double xv = (part[24 + ph] + part[ph]) + part[12 + ph];
          const double corr = bdot_ln12(Wr, xv, 0.0);
          double* const zk = &sh.u.it.xs[XSL<N>(k)][ph];
          const double zv = *zk;
          if (cl) *zk = k == S ? xv : zv - corr;
          STAMP(8);
        }
      };
      // the state sweep: the lagging form up to 32 stages, the split form beyond
      // (kND: the nested-dissection solve)
      auto ph_sweep = [&]() __attribute__((always_inline)) {
        if constexpr (kND<N>) {
          ph_sweep_nd(nullptr);
        } else if constexpr (BIG) {
          ph_sweep_split();
        } else {
          ph_sweep_lag(std::integral_constant<int, N>{}, std::integral_constant<int, 3>{}, std::false_type{},
                       (lds_cd*)&sh.u.it.bo[0][0], 12 * N, &sh.u.it.yv[0][0], &sh.u.it.xs[0][0], GHr,
                       (lds_cd*)&sh.Sm[0][0]);
        }
      };
      // (kKI) the state x_i = sum over the eight waves' partial products P[w][i] (in GH), always
      // in wave order, so every lane that reads a state gets the same bits
      auto ki_psum = [&](int i) __attribute__((always_inline)) -> double {
        lds_cd* const q = GHr + i;
        double v = q[0];
#pragma unroll
        for (int w = 1; w < 2 * NW; ++w) v += q[12 * N * w];
        return v;
      };
      // ri0: 1/rho of the own slot-0 row (the ADMM loop's, or polish's)
      auto ph_recover = [&](const RhsOps* op, double ri0, double uf, double beta, double& sf, double& sX,
                            double (&ax)[3], const RecPre* pre = nullptr)
          __attribute__((always_inline)) {
          // P8: forces f_k = F_k (b_f - R B' g) = u - (F W) g, with g = Xd X_{k+1} + Hd X_k
          // on the velocity rows (the states' part of those rows)
          double gv;
          MPCQ_LANE_OFFS(kRecompLoop);
          // the iteration-invariant LDS operands of P8 / P9 are read before the
          // barrier that ends the sweeps (their latency hides behind it), the
          // sweep's states after it (kND: read by ph_sweep_nd, pre)
          double fwl[6], qll[6], cFb, cFa, cF4;
          if constexpr (kND<N>) {
            RecPre own_;
            if (!pre) rec_pre(own_);
            const RecPre& q_ = pre ? *pre : own_;
#pragma unroll
            for (int i = 0; i < 6; ++i) { fwl[i] = q_.fwl[i]; qll[i] = q_.qll[i]; }
            cFb = q_.cFb; cFa = q_.cFa; cF4 = q_.cF4;
          } else {
#pragma unroll
            for (int i = 0; i < 3; ++i) {  // 16-B aligned pairs: ds_read_b128 (twice ds_read2_b64's LDS rate)
              using wcd2 = std::conditional_t<BIG, const dbl2, lds_cd2>;
              const dbl2 fa = ((lds_cd2*)(FWr + oFW))[i], qa = ((wcd2*)(QLr + oQLm))[i];
              fwl[2 * i] = fa.x; fwl[2 * i + 1] = fa.y;
              qll[2 * i] = qa.x; qll[2 * i + 1] = qa.y;
            }
          }
          // (the same coefficients as ph_rhs's, from the held set when there is one)
          const double eXd = op ? op->cXd : Ab[oXd], eHd = op ? op->cHd : Ab[oHdm], eH6 = op ? op->cH6 : Ab[oH6m];
          if constexpr (!kND<N>) { cFb = Ab[oFb]; cFa = Ab[oFa]; cF4 = Ab[oF4]; }
          const double cSw = op ? op->cf[4] : Ab[oF + 4];
          sync_all();
          STAMP(7);
          double xa, xb;
          if constexpr (KI) {  // the explicit inverse's product (stage 0: X_0 = 0)
            const int ip = 12 * (hp ? k - 1 : k);
            sX = ki_psum(12 * k + ph);
            const double a_ = ki_psum(ip + ph), b_ = ki_psum(ip + (ph < 6 ? ph + 6 : ph));
            xa = hp ? a_ : 0.0;
            xb = hp ? b_ : 0.0;
          } else {
            xa = XSr[rXSpm];  // (stage 0: X_0 = 0, a zero slot)
            xb = XSr[rXSp6m];
            sX = XSr[rXS];
          }
          asm volatile("" : : : "memory");
          {
            gv = eXd * sX + eHd * xa;  // used from the lanes of rows 6..11 only
            sf = uf - bdot_ln6v(fwl, gv, 0.0);
          }
          STAMP(9);
          // P9: z, y update (osqp update_z / update_y), x update.  A x~ on the own rows:
          // dynamics rows use B f = B u - B F W g = beta / rho - (R^{-1} Q) g (no force gather)
          {
            {
              // B f on the velocity rows (zero coefficients elsewhere)
              const double bfv = beta * ri0 - bdot_ln6v(qll, gv, 0.0);
              const double dyn = (gv + eH6 * xb) + bfv;
              // friction rows: lane c < 3 owns row c, lane 3 rows 3 and 4 (all loads unconditional)
              const double q0 = qbc<0>(sf), q1 = qbc<1>(sf), q2 = qbc<2>(sf);
              const double frA = cFb * q2 + cFa * (ta0 ? q0 : q1);
              const double frB = cF4 * q2;
              const double swg = cSw * sf;
              ax[0] = cl ? dyn : frA;
              ax[1] = cl ? swg : frB;
              ax[2] = cl ? frA : 0.0;
            }
          }
      };
      const double kNoW[3] = {0.0, 0.0, 0.0};

      // ---- (kKI) the explicit inverse Z = K_s^{-1}: formation and product ----------------
      using KL = KinvLay<N>;
      // the wave index as a wave-uniform (scalar) value: the roles and column ranges branch on it
      auto wvu = [&]() __attribute__((always_inline)) -> int { return __builtin_amdgcn_readfirstlane(t >> 6); };
      // the summed right-hand side of iteration parity b (kKI): u.it.nb (b = 0) / u.it.yv (b = 1),
      // free during the iterations (the checks publish there, then zero them again)
      auto ki_rsum = [&](int b_) __attribute__((always_inline)) -> lds_d* {
        return (lds_d*)(b_ ? &sh.u.it.yv[0][0] : &sh.u.it.nb[0][0]);
      };
      // One 16-column tile of Z (columns cb .. cb + 15) by the two-ended sweep on the
      // identity's columns, both chains in this wave, every block product a 16 x 16 x 12
      // MFMA (v_mfma_f64_16x16x4_f64 x 3).  Tiles in the D layout: lane l holds rows
      // (l >> 4) + 4 r, r = 0..3, of column l & 15 (rows 12..15 are zero); a result's register
      // s is the next product's B operand for K-slice s, so a chain step moves no data.
      // A operands: lane l supplies M[l & 15][4 s + (l >> 4)] (transposed: M[4 s + (l >> 4)][l & 15]).
      // The step's w = S^{-1} y tiles are parked in KV at the columns' own rows and read back
      // by the outward steps, which overwrite them with the results (the pass's staging):
      //   top    y_0 = e_0, y_k = e_k - G_k y_{k-1} (k <= MID), w_k = S_k^{-1} y_k (k < MID)
      //   bottom v_{N-1} = e_{N-1}, v_k = e_k - H_k v_{k+1} (k >= MID), w_k = U_k^{-1} v_k (k > MID)
      //   x_MID = M^{-1} (y_MID + v_MID - e_MID)
      //   x_k = w_k - G_{k+1}' x_{k+1} (k < MID),  x_k = w_k - H_{k-1}' x_{k-1} (k > MID)
      // (-G, -H are stored negated: every step is an accumulation.)
      auto ki_tile = [&](int c0, int cn, int cb) __attribute__((always_inline)) {
        const int l = lane, cc = l & 15, rb = l >> 4;
        const int c = cb + cc;                    // this lane's column of Z
        const bool keep = c < c0 + cn;            // columns past the pass are computed, not stored
        double* const col = &sh.KV[0] + KL::KVS * (keep ? c - c0 : 0) + rb;  // + 12 k + 4 r: row 12 k + rb + 4 r
        const dbl4 zero4 = {0.0, 0.0, 0.0, 0.0};
        auto e_of = [&](int kk) __attribute__((always_inline)) -> dbl4 {  // the identity's rows of stage kk
          dbl4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (r < 3 && 12 * kk + rb + 4 * r == c) ? 1.0 : 0.0;
          return v;
        };
        // acc + M x (M 12 x 12 row-major in LDS at q; tr: M') for a tile x in the D layout
        auto mm = [&](const double* q, bool tr, const dbl4& x, dbl4 acc) __attribute__((always_inline)) -> dbl4 {
#pragma unroll
          for (int s_ = 0; s_ < 3; ++s_) {
            const int o = tr ? 12 * (4 * s_ + rb) + cc : 12 * cc + 4 * s_ + rb;
            const double av = cc < 12 ? q[cc < 12 ? o : 0] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, x[s_], acc, 0, 0, 0);
          }
          return acc;
        };
        auto park = [&](int kk, const dbl4& v) __attribute__((always_inline)) {
          if (keep) {
#pragma unroll
            for (int r = 0; r < 3; ++r) col[12 * kk + 4 * r] = v[r];
          }
        };
        auto unpark = [&](int kk) __attribute__((always_inline)) -> dbl4 {
          dbl4 v = zero4;
          if (keep) {
#pragma unroll
            for (int r = 0; r < 3; ++r) v[r] = col[12 * kk + 4 * r];
          }
          return v;
        };
        const double* const smp = &sh.Sm[0][0];
        dbl4 yT = e_of(0), vB = e_of(N - 1);
        park(0, mm(smp + SLOT<N>(SIG<N>(0)), false, yT, zero4));
        park(N - 1, mm(smp + SLOT<N>(SIG<N>(N - 1)), false, vB, zero4));
#pragma unroll
        for (int kk = 1; kk <= MID; ++kk) {
          yT = mm(gh0 + SLOT<N>(SIG<N>(kk)), false, yT, e_of(kk));
          if (kk < MID) park(kk, mm(smp + SLOT<N>(SIG<N>(kk)), false, yT, zero4));
          const int kb = N - 1 - kk;
          if (kb >= MID) {
            vB = mm(gh0 + SLOT<N>(SIG<N>(kb + 1)), false, vB, e_of(kb));
            if (kb > MID) park(kb, mm(smp + SLOT<N>(SIG<N>(kb)), false, vB, zero4));
          }
        }
        const dbl4 em = e_of(MID);
        dbl4 t4;
#pragma unroll
        for (int r = 0; r < 4; ++r) t4[r] = (yT[r] + vB[r]) - em[r];
        const dbl4 xm = mm(gh0, false, t4, zero4);  // M^{-1} in GH slot 0
        park(MID, xm);
        dbl4 xT = xm, xB = xm;
#pragma unroll
        for (int j = 1; j <= (MID > N - 1 - MID ? MID : N - 1 - MID); ++j) {
          const int kt = MID - j, kb = MID + j;
          if (kt >= 0) {
            xT = mm(gh0 + SLOT<N>(SIG<N>(kt + 1)), true, xT, unpark(kt));
            park(kt, xT);
          }
          if (kb <= N - 1) {
            xB = mm(gh0 + SLOT<N>(SIG<N>(kb)), true, xB, unpark(kb));
            park(kb, xB);
          }
        }
      };
      // Z after a factorisation: four passes of at most 54 columns staged in KV (the last
      // pass is KV's own part); a helper copies the columns it owns from each staged pass.
      // Both roles run the same barriers.
      auto kinv_form = [&](auto role, double (&kv)[3 * KL::HC]) __attribute__((always_inline)) {
        constexpr bool H = decltype(role)::value;
        if constexpr (!H) {  // the summed right-hand sides start from zero (their barriers follow)
          if (cl) { ki_rsum(0)[12 * k + ph] = 0.0; ki_rsum(1)[12 * k + ph] = 0.0; }
        }
#pragma nounroll
        for (int q = 0; q < KL::NPASS; ++q) {
          const int c0 = KL::pc0(q), cn = KL::pcn(q);
          if constexpr (!H) {
            const int w_ = wvu();
            if (w_ * 16 < cn) ki_tile(c0, cn, c0 + 16 * w_);
          }
          sync_all();
          if constexpr (H) {
            if (q < KL::NPASS - 1) {
              const int h = wvu() - NW, hc = KL::hc0(h), hn = KL::hcn(h);
#pragma unroll
              for (int j = 0; j < KL::HC; ++j) {
                const int cj = hc + j;
                if (j < hn && cj >= c0 && cj < c0 + cn) {
                  const double* const src = &sh.KV[0] + KL::KVS * (cj - c0) + lane;
                  kv[3 * j] = src[0];
                  kv[3 * j + 1] = src[64];
                  kv[3 * j + 2] = src[128];
                }
              }
            }
          }
          sync_all();
        }
      };
      // x = Z r, r = bo + na (the state right-hand sides ph_rhs published): this wave's
      // columns times r into P[wave][row] (rows lane, lane + 64, lane + 128), in column order.
      // Helpers: their register columns; stage waves: their KV columns.
      // x = Z r: r is loaded once, distributed (lane s of every 16-lane row holds r of the
      // wave's column 16 u + s), and each column's three FMAs take it by row broadcast
      // (v_fmac_f64_dpp row_newbcast:s): no per-column LDS load.  Helpers multiply their
      // register columns; stage waves load their KV columns in two halves (all issued before
      // the first half's FMAs).  Three accumulation chains (rows lane, lane + 64, lane + 128),
      // each in column order.
      auto kinv_mv = [&](auto role, const double (&kv)[3 * KL::HC], lds_cd* const rs) __attribute__((always_inline)) {
        constexpr bool H = decltype(role)::value;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
        // (lane ids from a laundered thread index: held across the loop they were spilled)
        int tl_ = t;
        asm volatile("" : "+v"(tl_));
        const int ln_ = tl_ & 63, s16 = tl_ & 15;
        if constexpr (H) {
          const int h = wvu() - NW, hn = KL::hcn(h);
          lds_cd* const rq = rs + KL::hc0(h);  // (hc0 + 47 < 192: in the buffer)
          double rv[3];
#pragma unroll
          for (int u = 0; u < 3; ++u) rv[u] = rq[16 * u + s16];
          auto col = [&](auto jt) __attribute__((always_inline)) {
            constexpr int j = decltype(jt)::value;
            if (j < KL::HC - 1 || j < hn)
              fmac3_bc<j % 16>(a0, a1, a2, rv[j / 16], kv[3 * j], kv[3 * j + 1], kv[3 * j + 2]);
          };
          for_each_j(col, std::make_integer_sequence<int, KL::HC>{});
        } else {
          const int w_ = wvu(), sc = KL::sc0(w_), sn = KL::scn(w_);
          lds_cd* const kq = (lds_cd*)&sh.KV[0] + KL::KVS * (sc - KL::SP0) + ln_;
          const double rv = rs[sc + (s16 < sn ? s16 : 0)];
          constexpr int HALF = 7;
          double ka[3 * HALF], kb[3 * HALF];
#pragma unroll
          for (int i = 0; i < HALF; ++i) {
            const int ja = i, jb = HALF + i < sn ? HALF + i : sn - 1;  // (clamped: no read past KV)
            ka[3 * i] = kq[KL::KVS * ja]; ka[3 * i + 1] = kq[KL::KVS * ja + 64]; ka[3 * i + 2] = kq[KL::KVS * ja + 128];
            kb[3 * i] = kq[KL::KVS * jb]; kb[3 * i + 1] = kq[KL::KVS * jb + 64]; kb[3 * i + 2] = kq[KL::KVS * jb + 128];
          }
          asm volatile("" ::: "memory");
          auto col = [&](auto jt, const double (&kk)[3 * HALF]) __attribute__((always_inline)) {
            constexpr int j = decltype(jt)::value, i = j % HALF;
            if (j < 2 * HALF - 1 || j < sn) fmac3_bc<j>(a0, a1, a2, rv, kk[3 * i], kk[3 * i + 1], kk[3 * i + 2]);
          };
          for_each_j([&](auto jt) __attribute__((always_inline)) { col(jt, ka); }, std::make_integer_sequence<int, HALF>{});
          for_each_j([&](auto jt) __attribute__((always_inline)) {
            col(std::integral_constant<int, HALF + decltype(jt)::value>{}, kb);
          }, std::make_integer_sequence<int, HALF>{});
        }
        double* const P = gh0 + 12 * N * wvu() + ln_;
        P[0] = a0;
        P[64] = a1;
        P[128] = a2;
      };

      // ------------------------------------------------------------ ADMM
      // The factorisation sits outside the hot loop: the outer loop factors,
      // the inner loop iterates until convergence, max_iter or a rho update.
      bool last_checked = false;
      int iter = 1;
      // the loop's exit status: LDS (kXstLds; read after the loop's closing barrier) or status
#define MPCQ_SET_XST(v_) do { if constexpr (kXstLds<N>) { if (t == 0) sh.flag[4] = (v_); } else if constexpr (!kXstRe<N>) { status = (v_); } } while (0)
      if constexpr (kXstLds<N>) MPCQ_SET_XST(0);
      int to_check = p.check_termination, to_adapt = p.adaptive_rho_interval;
      if constexpr (KI) {
        // (kKI) the loop of the explicit inverse: one driver for both roles, the helpers
        // (waves NW..) with std::true_type -- the same barriers and the same uniform
        // decisions (info_combine reads the stage waves' partials from LDS), no stage work
        auto kinv_admm = [&](auto role) __attribute__((always_inline)) {
          constexpr bool H = decltype(role)::value;
          double kv[3 * KL::HC];  // (helpers) Z's columns hc0.. : rows lane, lane + 64, lane + 128
#pragma unroll
          for (int j = 0; j < 3 * KL::HC; ++j) kv[j] = 0.0;
          const bool chk_on = p.check_termination > 0;
          const bool adp_on = p.adaptive_rho && p.adaptive_rho_interval > 0;
          for (;;) {
            if (!factor(role, p.sigma, nullptr)) { MPCQ_SET_XST(MPCQ_STATUS_FACTOR_FAILED); break; }
            kinv_form(role, kv);
            STAMP(2);
            bool refactor = false;
            // one ADMM iteration: ph_rhs, barrier A, the product, ph_recover (barrier B), update
            auto ki_iter = [&](auto mode_tag, const RhsOps& ops, double (&dyv)[3], double& dxf_, double& dxX_,
                               double (&cvp)[CK_COUNT]) __attribute__((always_inline)) {
              constexpr bool DELTA = decltype(mode_tag)::value == 1;
              lds_d* const rs = ki_rsum(iter & 1);
              if constexpr (H) {
                STAMP(15);
                sync_all();  // A
                STAMP(3);
                kinv_mv(role, kv, rs);
                if constexpr (DELTA) ck_all(cvp);
                STAMP(6);
                sync_all();  // B
                STAMP(7);
              } else {
                double uf, beta, sf, sX, ax[3];
                ph_rhs(true, &ops, kNoW, 0.0, 0.0, uf, beta, rs);
                STAMP(15);
                sync_all();  // A: r = bo + na summed
                STAMP(3);
                kinv_mv(role, kv, rs);
                STAMP(6);
                if constexpr (DELTA) ck_all(cvp);
                ph_recover(&ops, ri[0], uf, beta, sf, sX, ax);  // (B inside: the partial products)
                // every read of this buffer preceded B; it is summed into again two iterations on
                if (cl) rs[12 * k + ph] = 0.0;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                  const double zr = p.alpha * ax[j] + (1.0 - p.alpha) * z[j];
                  const double tt = zr + ri[j] * y[j];
                  const double zn = fmin(fmax(tt, lo_of(j)), hi_of(j));  // osqp project
                  const double d = rr[j] * (zr - zn);
                  if constexpr (DELTA) dyv[j] = d;
                  y[j] = y[j] + d;
                  z[j] = zn;
                }
                const double nxf = p.alpha * sf + (1.0 - p.alpha) * xf;
                const double nxX = p.alpha * sX + (1.0 - p.alpha) * xX;
                if constexpr (DELTA) { dxf_ = nxf - xf; dxX_ = nxX - xX; }
                xf = nxf;
                xX = nxX;
              }
              STAMP(10);
            };
            while (iter <= p.max_iter) {
              int until = p.max_iter - iter + 1;
              if (chk_on && to_check < until) until = to_check;
              if (adp_on && to_adapt < until) until = to_adapt;
              double dyv[3], dxf_, dxX_;
              RhsOps ops;
              if constexpr (!H) load_rhs_ops(ops);
              double cvp[CK_COUNT];
#pragma nounroll
              for (int r_ = 1; r_ < until; ++r_, ++iter)
                ki_iter(std::integral_constant<int, 0>{}, ops, dyv, dxf_, dxX_, cvp);
              ki_iter(std::integral_constant<int, 1>{}, ops, dyv, dxf_, dxX_, cvp);
              const bool can_check = chk_on && (to_check -= until) == 0;
              if (can_check) to_check = p.check_termination;
              const bool adapt = adp_on && (to_adapt -= until) == 0;
              if (adapt) to_adapt = p.adaptive_rho_interval;
              last_checked = can_check;
              if constexpr (H) {
                sync_all();  // infeas_cheap's publication
                sync_all();  // update_info: the stage waves' residual terms
                info_combine(std::true_type{}, cvp, sh.red, 32);
                sync_all();
              } else {
                infeas_cheap(dyv, dxf_, dxX_, cvp);
                update_info(std::true_type{}, cvp);
              }
              if (inf_need) infeas_products(role, dxf_, dxX_, cvp);
              // the checks published into the summed right-hand sides' buffers: zero them again,
              // and a barrier before the next iteration sums into them
              if constexpr (!H) {
                if (cl) { ki_rsum(0)[12 * k + ph] = 0.0; ki_rsum(1)[12 * k + ph] = 0.0; }
              }
              sync_all();
              if (!(isfinite(pri_res) && isfinite(dua_res))) { MPCQ_SET_XST(MPCQ_STATUS_NONFINITE); break; }
              if (can_check) {
                if (converged(1.0)) { MPCQ_SET_XST(MPCQ_STATUS_SOLVED); break; }
                if (inf_bits & 1) { MPCQ_SET_XST(MPCQ_STATUS_PRIMAL_INFEASIBLE); break; }
                if (inf_bits & 2) { MPCQ_SET_XST(MPCQ_STATUS_DUAL_INFEASIBLE); break; }
              }
              if (adapt) {
                double rn = rho_s * sqrt(s_pri / (s_dua + kDivTol));
                rn = fmin(fmax(rn, kRhoMin), kRhoMax);
                if (rn > rho_s * p.adaptive_rho_tolerance || rn < rho_s / p.adaptive_rho_tolerance) {
                  rho_s = rn;
                  if constexpr (!H) {
                    set_rho();
                    zc_store();
                  }
                  refactor = true;
                  ++n_upd;
                  ++iter;
                  sync_all();
                  break;
                }
              }
              STAMP(11);
              ++iter;
            }
            if (!refactor) break;
          }
          sync_all();  // thread 0's exit status (kXstLds)
          if constexpr (!H) status = sh.flag[4];
        };
        static_assert(!KI || kXstLds<N>, "the explicit inverse reads the exit status from LDS");
        if (wvu() >= NW) {  // the helpers: nothing of theirs is an output
          kinv_admm(std::true_type{});
          return;
        }
        kinv_admm(std::false_type{});
      } else {
      // a resumed slice continues the saved loop counters; slice_iters > 0 suspends at the
      // first segment end slice_iters iterations on (mpcq_set_slice)
      if (kSlice<N> && a.resume) {
        iter = __builtin_amdgcn_readfirstlane(a.res_i[8 * b]);
        to_check = __builtin_amdgcn_readfirstlane(a.res_i[8 * b + 1]);
        to_adapt = __builtin_amdgcn_readfirstlane(a.res_i[8 * b + 2]);
      }
      const int slice_end =
          kSlice<N> && a.slice_iters > 0 && a.slice_iters < p.max_iter ? iter + a.slice_iters : 0x7fffffff;
      bool suspended = false;
      // the bounds are re-derived where used (lo_of / hi_of: a select on the lane's
      // class and its row scaling in the fused path) rather than held in 6 registers
      for (;;) {
#ifndef MPCQ_REP_FACTOR
#define MPCQ_REP_FACTOR 1
#endif
        bool fac_ok = true;
#ifdef MPCQ_FACTIME
        const uint64_t ft0_ = __builtin_amdgcn_s_memtime();
#endif
#pragma nounroll
        for (int rep_ = 0; rep_ < MPCQ_REP_FACTOR; ++rep_) fac_ok = factor(std::false_type{}, p.sigma, nullptr);  // > 1: timing only
#ifdef MPCQ_FACTIME
        fac_cycles += __builtin_amdgcn_s_memtime() - ft0_;
#endif
        if (!fac_ok) { MPCQ_SET_XST(MPCQ_STATUS_FACTOR_FAILED); break; }
        STAMP(2);
        bool refactor = false;
        // One ADMM iteration (osqp update_xz_tilde / update_x / update_z / update_y).
        // DELTA: also keep delta_y / delta_x (the last iteration before a check, for the
        // infeasibility tests).  The iterations between two checks run in a loop of
        // their own without them, so the check / infeasibility code and its live values
        // sit outside the hot loop's register allocation (inside it, they cost 0.31 us
        // per iteration through spills on the sweep path, measured).
        // MODE 0: a plain iteration; 1 (DELTA): the checked one, also keeping delta_y / delta_x
        auto admm_iter = [&](auto mode_tag, const RhsOps& ops, double (&dyv)[3], double& dxf_, double& dxX_,
                             double (&cvp)[CK_COUNT])
            __attribute__((always_inline)) {
          constexpr int MODE = decltype(mode_tag)::value;
          constexpr bool DELTA = MODE == 1;
          double uf, beta, sf, sX, ax[3];
          // (beyond 32 stages the operands are read per iteration: held, they cost the
          // register budget of the 9..16-wave workgroups -- N = 48: scratch 840 -> 712 B
          // per lane, 17.68 -> 16.75 us per iteration, profiles/r03c_iterbench.txt)
          ph_rhs(true, kBig<N> ? nullptr : &ops, kNoW, 0.0, 0.0, uf, beta);
          [[maybe_unused]] RecPre pre_;
          if constexpr (kND<N>) ph_sweep_nd(&pre_);
          else ph_sweep();
          // DELTA (the last iteration before a check): the check's constant block is read
          // here, its memory latency behind the force recovery and the z / y / x update
          if constexpr (DELTA) ck_all(cvp);
          double zl[3], zh[3], zrr[3], zri[3];  // the update's per-row constants
          if constexpr (kZcMem<N>) {
            ph_recover(nullptr, zc_ptr()[ZC_RI], uf, beta, sf, sX, ax);
            pdbl* const q = zc_ptr();
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              zl[j] = q[ZC_LO + j]; zh[j] = q[ZC_HI + j]; zrr[j] = q[ZC_RR + j]; zri[j] = q[ZC_RI + j];
            }
          } else {
            ph_recover(kBig<N> ? nullptr : &ops, ri[0], uf, beta, sf, sX, ax, kND<N> ? &pre_ : nullptr);
#pragma unroll
            for (int j = 0; j < 3; ++j) { zl[j] = lo_of(j); zh[j] = hi_of(j); zrr[j] = rr[j]; zri[j] = ri[j]; }
          }
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const double zr = p.alpha * ax[j] + (1.0 - p.alpha) * z[j];
            const double tt = zr + zri[j] * y[j];
            const double zn = clamp_hw(tt, zl[j], zh[j]);  // osqp project: c_min(c_max(tt, l), u)
            const double d = zrr[j] * (zr - zn);
            if constexpr (DELTA) dyv[j] = d;
            y[j] = y[j] + d;
            z[j] = zn;
          }
          const double nxf = p.alpha * sf + (1.0 - p.alpha) * xf;
          const double nxX = p.alpha * sX + (1.0 - p.alpha) * xX;
          if constexpr (DELTA) { dxf_ = nxf - xf; dxX_ = nxX - xX; }
          xf = nxf;
          xX = nxX;
          STAMP(10);
        };
        const bool chk_on = p.check_termination > 0;
        const bool adp_on = p.adaptive_rho && p.adaptive_rho_interval > 0;
        while (iter <= p.max_iter) {
          // the next event: a termination check, an adaptive-rho step or the last iteration
          int until = p.max_iter - iter + 1;
          if (chk_on && to_check < until) until = to_check;
          if (adp_on && to_adapt < until) until = to_adapt;
          double dyv[3], dxf_, dxX_;
          // held in registers through the iterations up to the next check: no LDS traffic
          // for them in the loop
          RhsOps ops;
          if constexpr (!kBig<N>) load_rhs_ops(ops);
          double cvp[CK_COUNT];
#pragma nounroll
          for (int r_ = 1; r_ < until; ++r_, ++iter)
            admm_iter(std::integral_constant<int, 0>{}, ops, dyv, dxf_, dxX_, cvp);
          admm_iter(std::integral_constant<int, 1>{}, ops, dyv, dxf_, dxX_, cvp);
          // iter % check_termination == 0 / iter % adaptive_rho_interval == 0, by countdown
          const bool can_check = chk_on && (to_check -= until) == 0;
          if (can_check) to_check = p.check_termination;
          const bool adapt = adp_on && (to_adapt -= until) == 0;
          if (adapt) to_adapt = p.adaptive_rho_interval;
          last_checked = can_check;
          // the last iteration's information is always formed here, while its deltas are
          // live (osqp's update_info after the loop when the last iteration was unchecked)
          infeas_cheap(dyv, dxf_, dxX_, cvp);
          update_info(std::true_type{}, cvp);
          if (inf_need) infeas_products(std::false_type{}, dxf_, dxX_, cvp);
          if (!(isfinite(pri_res) && isfinite(dua_res))) { MPCQ_SET_XST(MPCQ_STATUS_NONFINITE); break; }
          if (can_check) {  // osqp check_termination
            if (converged(1.0)) { MPCQ_SET_XST(MPCQ_STATUS_SOLVED); break; }
            if (inf_bits & 1) { MPCQ_SET_XST(MPCQ_STATUS_PRIMAL_INFEASIBLE); break; }
            if (inf_bits & 2) { MPCQ_SET_XST(MPCQ_STATUS_DUAL_INFEASIBLE); break; }
          }
          if (adapt) {
            double rn = rho_s * sqrt(s_pri / (s_dua + kDivTol));
            rn = fmin(fmax(rn, kRhoMin), kRhoMax);
            if (rn > rho_s * p.adaptive_rho_tolerance || rn < rho_s / p.adaptive_rho_tolerance) {
              rho_s = rn;
              set_rho();
              zc_store();
              refactor = true;
              ++n_upd;
              ++iter;
              sync_all();
              break;
            }
          }
          STAMP(11);
          ++iter;
          // (a sliced launch) the residuals over their tolerances at the last segment end up to
          // half way through the slice, for the suspended instance's key (below)
          if (kSlice<N> && a.slice_iters > 0 && iter <= slice_end - (a.slice_iters >> 1) && t == 0) {
            a.res_key[2 * b] = pri_res / eps_pri;
            a.res_key[2 * b + 1] = dua_res / eps_dua;
            a.res_i[8 * b + 4] = iter;
          }
          if (kSlice<N> && iter >= slice_end && iter <= p.max_iter) {  // (uniform) suspend this slice here
            suspended = true;
            break;
          }
        }
        if (!refactor) break;
      }
      if (kSlice<N> && suspended) {  // the iterate and the loop's counters for the next slice; no other output
        constexpr int64_t RL = res_lanes(N);
        double* const q = a.res + b * 8 * RL + t;
        q[0] = xf;
        q[RL] = xX;
#pragma unroll
        for (int j = 0; j < 3; ++j) { q[(2 + j) * RL] = z[j]; q[(5 + j) * RL] = y[j]; }
        if (t == 0) {
          a.res_rho[b] = rho_s;
          // the key: the iterations left, extrapolated from the residuals' geometric decay between
          // the half-way sample and now, primal and dual, the larger (a residual not decaying, or
          // no half-way sample: as long as can be); 0 for one already within its tolerance
          const int i1 = a.res_i[8 * b + 4];
          const double rp = pri_res / eps_pri, rd = dua_res / eps_dua;
          auto left = [&](double r1, double r2) __attribute__((always_inline)) -> double {
            if (!(r2 > 1.0)) return 0.0;
            if (i1 <= 0 || !(r1 > r2)) return 1e30;
            return log(r2) / log(r1 / r2) * (double)(iter - i1);
          };
          a.res_key[2 * b] = fmax(left(a.res_key[2 * b], rp), left(a.res_key[2 * b + 1], rd));
          a.res_i[8 * b] = iter;
          a.res_i[8 * b + 1] = to_check;
          a.res_i[8 * b + 2] = to_adapt;
          a.res_i[8 * b + 3] = n_upd;
          if (a.status) a.status[b] = kStatusSuspended;
        }
        return;
      }
      if constexpr (kXstLds<N>) {
        sync_all();  // thread 0's exit status
        status = sh.flag[4];
      }
      }  // !KI
      if constexpr (kXstRe<N>) {  // the exit's reason, as the loop tested it (kXstRe)
        if (sh.flag[2] != 0) status = MPCQ_STATUS_FACTOR_FAILED;
        else if (iter <= p.max_iter) {
          if (!(isfinite(pri_res) && isfinite(dua_res))) status = MPCQ_STATUS_NONFINITE;
          else if (converged(1.0)) status = MPCQ_STATUS_SOLVED;
          else if (inf_bits & 1) status = MPCQ_STATUS_PRIMAL_INFEASIBLE;
          else if (inf_bits & 2) status = MPCQ_STATUS_DUAL_INFEASIBLE;
        }
      }
#undef MPCQ_SET_XST
      it_done = iter > p.max_iter ? p.max_iter : iter;
      if (status == 0) {
        if (!last_checked) {  // the information of the last (unchecked) iteration
          if (converged(1.0)) status = MPCQ_STATUS_SOLVED;
          else if (inf_bits & 1) status = MPCQ_STATUS_PRIMAL_INFEASIBLE;
          else if (inf_bits & 2) status = MPCQ_STATUS_DUAL_INFEASIBLE;
        }
        if (status == 0)  // the approximate check (tolerances x10)
          status = converged(10.0) ? MPCQ_STATUS_SOLVED_INACCURATE
                   : (inf_bits & 4) ? MPCQ_STATUS_PRIMAL_INFEASIBLE_INACCURATE
                   : (inf_bits & 8) ? MPCQ_STATUS_DUAL_INFEASIBLE_INACCURATE
                                   : MPCQ_STATUS_MAX_ITER_REACHED;
      }

      admm_st = status;
      // ------------------------------------------------------------ polish
      // OSQP 0.6 polish (polish.c): guess the active set from (z, y), solve the
      // equality-constrained QP  min 1/2 x'Px  s.t. A_act x = b_act,  project
      // (A x, y) onto the normal cone and keep the point if it lowers the
      // residuals; polish_rounds > 1 repeats the guess from the polished point
      // until the set repeats (primal-dual active set).  The equality QP is solved
      // by the method of multipliers on the engine's own factorisation
      // (K = P + sigma I + rho_p A_act' A_act, rho_p = kPolishRho):
      //   x+ = K^{-1} (sigma x + A_act' (rho_p b - y)),  y+ = y + rho_p (A_act x+ - b),
      // 1 + max(polish_refine_iter, kPolishMinIter) solves.  OSQP's own reduced KKT
      // (rho = 1/delta = 1e6) is not used: the engine's stage elimination forms
      // F = K_ff^{-1} explicitly, and at 1e6 its Schur complements lose positive
      // definiteness (measured: negative pivots on every instance).  Equality rows
      // stay in the set even when y is exactly 0.
      if constexpr (POLISH) {
        if (p.polish != 0 && (status == MPCQ_STATUS_SOLVED ||
                              (p.polish >= 2 && (status == MPCQ_STATUS_SOLVED_INACCURATE ||
                                                 status == MPCQ_STATUS_MAX_ITER_REACHED)))) {
          constexpr double kPolishRho = 1e3;
          // the refinement contracts by the error of the explicit stage inverses, which
          // grows with the chain length: 10 steps land within 2e-10 of x* up to N = 32,
          // N = 48 needs 20 (measured: 10 -> 2-4e-7, 20 -> 1e-10, tools/attic/polish48b.py),
          // N = 64 more than 20 (20 -> 3.2e-8 on the fixtures, r03b)
          constexpr int kPolishMinIter = N > 48 ? 30 : (N > 32 ? 20 : 10);
          const double a_pri = pri_res, a_dua = dua_res;
          const double axf = xf, axX = xX;
          double az[3], ay[3], zs[3], ys[3], bred[3], prho[3];
          int act[3], prv[3];
#pragma unroll
          for (int j = 0; j < 3; ++j) { az[j] = z[j]; ay[j] = y[j]; zs[j] = z[j]; ys[j] = y[j]; prv[j] = 0; }
          bool have = false;
          double b_pri = 0.0, b_dua = 0.0, b_epri = 0.0, b_edua = 0.0, bxf = 0.0, bxX = 0.0, bz[3], by[3];
          const int rounds = p.polish_rounds > 0 ? p.polish_rounds : 1;
          const int mom = p.polish_refine_iter > kPolishMinIter ? p.polish_refine_iter : kPolishMinIter;
          for (int rd = 0; rd < rounds; ++rd) {
            int changed = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const int r = nat_row(j);
              const bool eq = ((cls >> (2 * j)) & 3u) == RC_EQ;
              int a_ = 0;
              if (r >= 0) {
                if (rd == 0) {  // OSQP's guess (polish.c form_Ared)
                  if (zs[j] - lo_of(j) < -ys[j]) a_ = -1;
                  else if (hi_of(j) - zs[j] < ys[j]) a_ = 1;
                  if (eq && a_ == 0) a_ = 1;
                } else {  // keep correctly signed active rows, add violated rows
                  const double tol = 1e-12;
                  if (prv[j] == -1 && (ys[j] <= tol || eq)) a_ = -1;
                  else if (prv[j] == 1 && (ys[j] >= -tol || eq)) a_ = 1;
                  else if (zs[j] < lo_of(j) - tol) a_ = -1;
                  else if (zs[j] > hi_of(j) + tol) a_ = 1;
                }
              }
              changed |= a_ != prv[j];
              act[j] = a_;
              prv[j] = a_;
              bred[j] = a_ < 0 ? lo_of(j) : (a_ > 0 ? hi_of(j) : 0.0);
              prho[j] = a_ ? kPolishRho : 0.0;
            }
            if (rd > 0) {  // stop when the set repeats (uniform over the block)
              if (t == 0) sh.flag[3] = 0;
              sync_all();
              if (changed) atomicOr(&sh.flag[3], 1);
              sync_all();
              const bool same = sh.flag[3] == 0;
              sync_all();
              if (same) break;
            }
            ++pol_rounds;
            if (!factor(std::false_type{}, p.sigma, prho)) break;
#pragma unroll
            for (int j = 0; j < 3; ++j) { rr[j] = prho[j]; ri[j] = act[j] ? 1.0 / kPolishRho : 0.0; }
            // one proximal multiplier step from the ADMM point (x, y on the active rows),
            // then refinement against the true residuals of the equality QP
            //   r_x = -(P x + A_act' y),  r_y = b - A_act x,
            //   dx = K^{-1} (r_x + rho_p A_act' r_y),  dy = rho_p (A_act dx - r_y),
            // so that the error of the explicit stage inverses does not reach the fixed point
            double xpf, xpX, axp[3], yp[3];
            {
              double pw[3], uf, beta, ax[3];
#pragma unroll
              for (int j = 0; j < 3; ++j) {
                yp[j] = act[j] ? y[j] : 0.0;
                pw[j] = act[j] ? kPolishRho * bred[j] - yp[j] : 0.0;
              }
              ph_rhs(false, nullptr, pw, p.sigma * xf, p.sigma * xX, uf, beta);
              ph_sweep();
              ph_recover(nullptr, ri[0], uf, beta, xpf, xpX, ax);
#pragma unroll
              for (int j = 0; j < 3; ++j) {
                axp[j] = ax[j];
                if (act[j]) yp[j] += kPolishRho * (ax[j] - bred[j]);
              }
            }
            for (int it_ = 0; it_ < mom; ++it_) {
              double pw[3], ry[3], uf, beta, dxf, dxX, ax[3];
#pragma unroll
              for (int j = 0; j < 3; ++j) {
                ry[j] = act[j] ? bred[j] - axp[j] : 0.0;
                pw[j] = act[j] ? kPolishRho * ry[j] - yp[j] : 0.0;
              }
              ph_rhs(false, nullptr, pw, -Pbf() * xpf, -PbX() * xpX, uf, beta);
              ph_sweep();
              ph_recover(nullptr, ri[0], uf, beta, dxf, dxX, ax);
              xpf += dxf;
              xpX += dxX;
#pragma unroll
              for (int j = 0; j < 3; ++j) {
                axp[j] += ax[j];
                if (act[j]) yp[j] += kPolishRho * (ax[j] - ry[j]);
              }
#ifdef MPCQ_DEBUG_POLISH
              {
                double rmax = 0.0, dxm = fmax(fabs(dxf), fabs(dxX));
                for (int j = 0; j < 3; ++j) if (act[j]) rmax = fmax(rmax, fabs(axp[j] - bred[j]));
                for (int o = 32; o > 0; o >>= 1) { rmax = fmax(rmax, __shfl_xor(rmax, o)); dxm = fmax(dxm, __shfl_xor(dxm, o)); }
                if (b == 0 && lane == 0) printf("blk0 wave %d rd %d it %d max|Ax-b| %.3e max|dx| %.3e\n", wv, rd, it_, rmax, dxm);
              }
#endif
            }
            // the next round guesses from the unprojected point
#pragma unroll
            for (int j = 0; j < 3; ++j) { zs[j] = axp[j]; ys[j] = yp[j]; }
            // project onto the normal cone (polish.c project_normalcone), residuals
            xf = xpf;
            xX = xpX;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const double tt = axp[j] + yp[j];
              const double zz = fmin(fmax(tt, lo_of(j)), hi_of(j));
              z[j] = zz;
              y[j] = tt - zz;
            }
#ifdef MPCQ_DEBUG_POLISH
            if (b == 0)
              for (int j = 0; j < 3; ++j)
                if (fabs(y[j] - yp[j]) > 1e-9 || (act[j] == 0 && fabs(axp[j] - z[j]) > 1e-12))
                  printf("blk0 k %d s %d j %d row %d act %d bred %.3e ax %.6e yp %.3e -> z %.6e y %.3e lo %.3e hi %.3e\n",
                         k, s, j, nat_row(j), act[j], bred[j], axp[j], yp[j], z[j], y[j], lo_of(j), hi_of(j));
#endif
            {
              double cvq[CK_COUNT];
              ck_all(cvq);
              update_info(std::false_type{}, cvq);
            }
#ifdef MPCQ_DEBUG_POLISH
            if (b < 2 && t == 0) printf("blk %d rd %d admm pri %.3e dua %.3e | polished pri %.3e dua %.3e eps %.3e %.3e\n", (int)b, rd, a_pri, a_dua, pri_res, dua_res, eps_pri, eps_dua);
#endif
            if (!have || fmax(pri_res, dua_res) < fmax(b_pri, b_dua)) {
              have = true;
              b_pri = pri_res; b_dua = dua_res; b_epri = eps_pri; b_edua = eps_dua;
              bxf = xf; bxX = xX;
#pragma unroll
              for (int j = 0; j < 3; ++j) { bz[j] = z[j]; by[j] = y[j]; }
            }
          }
          const bool good = have && ((b_pri < a_pri && b_dua < a_dua) || (b_pri < a_pri && a_dua < 1e-10) ||
                                     (b_dua < a_dua && a_pri < 1e-10));
          if (good) {
            xf = bxf;
            xX = bxX;
#pragma unroll
            for (int j = 0; j < 3; ++j) { z[j] = bz[j]; y[j] = by[j]; }
            pol_st = 1;
            if (status != MPCQ_STATUS_SOLVED && b_pri < b_epri && b_dua < b_edua) status = MPCQ_STATUS_SOLVED;
          } else {
            xf = axf;
            xX = axX;
#pragma unroll
            for (int j = 0; j < 3; ++j) { z[j] = az[j]; y[j] = ay[j]; }
            pol_st = have ? -1 : 0;
          }
        }
      }
    }
    // ------------------------------------------------------------ outputs
    // osqp store_solution: no solution (x = y = NaN) for the infeasibility statuses
    const bool nan_out = status == MPCQ_STATUS_NONFINITE || status == MPCQ_STATUS_FACTOR_FAILED ||
                         status == MPCQ_STATUS_BAD_GAIT || status == MPCQ_STATUS_BAD_BOUNDS ||
                         status == MPCQ_STATUS_PRIMAL_INFEASIBLE ||
                         status == MPCQ_STATUS_DUAL_INFEASIBLE || status == MPCQ_STATUS_PRIMAL_INFEASIBLE_INACCURATE ||
                         status == MPCQ_STATUS_DUAL_INFEASIBLE_INACCURATE;
    if (cl) {
      const double vf = nan_out ? NAN : Df * xf, vX = nan_out ? NAN : DX * xX;
      if (a.x) { a.x[b * n + colF] = vf; a.x[b * n + colX] = vX; }
      if (a.f0 && k == 0) a.f0[b * 12 + ph] = vf;
    }
    if (a.y) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int r = nat_row(j);
        // dual_warm = 1: the scaled workspace y, what the next tick's warm start reads
        if (r >= 0) a.y[b * m + r] = nan_out ? NAN : (p.dual_warm ? y[j] : E[j] * y[j] / cscale);
      }
    }
#ifdef MPCQ_STAMPS
    STAMP(12);
    if (t == kStampT && a.stamps) {
      for (int i = 0; i < 16; ++i) a.stamps[b * 16 + i] = st_acc[i];
    }
#endif
    if (t == 0) {
      if (a.status) a.status[b] = status;
      if (a.iters) a.iters[b] = it_done;
      if (a.rho_out) a.rho_out[b] = rho_s;
      if (a.info) {
        a.info[4 * b + 0] = n_upd;
        a.info[4 * b + 1] = pol_st;
#ifdef MPCQ_FACTIME
        a.info[4 * b + 2] = (int)(fac_cycles >> 8);  // factorisation cycles / 256 (timing build)
#else
        a.info[4 * b + 2] = pol_rounds;
#endif
        a.info[4 * b + 3] = admm_st != 0 ? admm_st : status;  // the ADMM's exit status before polish
      }
    }
  }
}

template <int N>
hipError_t launch_t(bool fused, bool solve, const mpcq_params& p, const LaunchArgs& a,
                    hipStream_t s) {
  const dim3 grid((unsigned)a.batch), block(16 * kRows<N>), block2(16 * kRows<N> * (kKinv<N> ? 2 : 1));
  if ((kBig<N> || kND<N>) && solve && !a.work) return hipErrorInvalidValue;  // the caller sizes it with work_doubles(N)
  // polish lives in its own instantiation: the production kernel's code (and its
  // register allocation in the ADMM loop) does not carry it
  const bool pol = p.polish != 0;
  if (!solve) hipLaunchKernelGGL((engine_kernel<N, true, false, false>), grid, block, 0, s, p, a);
  else if (fused && pol) hipLaunchKernelGGL((engine_kernel<N, true, true, true>), grid, block, 0, s, p, a);
  else if (fused) hipLaunchKernelGGL((engine_kernel<N, true, true, false>), grid, block2, 0, s, p, a);
  else if (pol) hipLaunchKernelGGL((engine_kernel<N, false, true, true>), grid, block, 0, s, p, a);
  else hipLaunchKernelGGL((engine_kernel<N, false, true, false>), grid, block2, 0, s, p, a);
  return hipGetLastError();
}

}  // namespace

// One translation unit per horizon (the Makefile compiles this file once per
// N with -DMPCQ_ENGINE_N=N, in parallel); mpcq_dispatch.cpp picks the unit.
#ifndef MPCQ_ENGINE_N
#error "compile mpcq_engine.hip with -DMPCQ_ENGINE_N=<horizon> (see the Makefile)"
#endif
static_assert(MPCQ_ENGINE_N >= 4 && kRows<MPCQ_ENGINE_N> <= 64, "horizons 4..64 (1024 threads at most)");
static_assert(sizeof(Smem<MPCQ_ENGINE_N>) <= 160 * 1024, "Smem<N> exceeds the CU's LDS");
static_assert(sizeof(Smem<MPCQ_ENGINE_N, kKinv<MPCQ_ENGINE_N>>) <= 160 * 1024, "Smem<N, KI> exceeds the CU's LDS");
static_assert(Work<MPCQ_ENGINE_N>::SIZE == ((kBig<MPCQ_ENGINE_N> || kND<MPCQ_ENGINE_N>) ? work_doubles(MPCQ_ENGINE_N)
                                                                                   : 72 + Work<MPCQ_ENGINE_N>::ZERO),
              "work_doubles(N) (mpcq_internal.h) and Work<N> disagree");
static_assert(kRows<MPCQ_ENGINE_N> > 16 || sizeof(Smem<MPCQ_ENGINE_N>) <= 80 * 1024,
              "Smem<N> must fit twice in a CU for N <= 16");

#define MPCQ_CAT_(a, b) a##b
#define MPCQ_CAT(a, b) MPCQ_CAT_(a, b)
hipError_t MPCQ_CAT(engine_launch_n, MPCQ_ENGINE_N)(bool fused, bool solve, const mpcq_params& p,
                                                   const LaunchArgs& a, hipStream_t s) {
  return launch_t<MPCQ_ENGINE_N>(fused, solve, p, a, s);
}

}  // namespace mpcq
