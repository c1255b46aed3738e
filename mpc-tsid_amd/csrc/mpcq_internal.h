// mpcq_internal.h — shared between the HIP kernels and the host C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mpcq.h"

namespace mpcq {

// Per-launch arguments.  Every pointer is a device pointer.  Optional arrays
// may be null.  Layouts are the ones documented in include/mpcq.h.
struct LaunchArgs {
  int64_t batch;
  int mode;            // formulation mode (fused path)
  const double* xref;  // [B][12][N+1]   (fused / formulate)
  const double* fsteps;// [B][20][13]    (fused / formulate)
  const double* Ax;    // [B][nnz]       (qp path)
  const double* l;     // [B][m]         (qp path)
  const double* u;     // [B][m]         (qp path)
  const double* warm_x;// [B][n]
  const double* warm_y;// [B][m]
  const double* rho_in;// [B]
  double* Ax_out;      // [B][nnz]       (formulate)
  double* l_out;       // [B][m]
  double* u_out;       // [B][m]
  double* f0;          // [B][12]
  double* x;           // [B][n]
  double* y;           // [B][m]
  int32_t* status;     // [B]
  int32_t* iters;      // [B]
  double* rho_out;     // [B]
  int32_t* info;       // [B][4]: rho updates, polish status, polish rounds, reserved
  uint64_t* stamps;    // [B][16] diagnostic build only (MPCQ_STAMPS): cycles per phase
  double* work;        // [B][work_doubles(N)] engine workspace (N > 32 and the nested-dissection horizons)
  const int32_t* order; // [B] instance solved by workgroup i (a permutation of 0..B-1), or null: i
  // sliced solves (mpcq_set_slice): slice_iters > 0 suspends an instance at the first segment
  // end (a check / adaptive-rho / max_iter boundary of the ADMM loop) after slice_iters more
  // iterations: its iterate and loop counters to res / res_rho / res_i, status
  // kStatusSuspended, no other output.  resume != 0: every instance of this launch starts from
  // its saved iterate (the formulation, scaling and factorisation at the saved rho recomputed:
  // the same bits) instead of the cold point.
  int32_t slice_iters;
  int32_t resume;
  const int32_t* batch_dev;  // (the resumed launch) the count of workgroups with work, on the device:
                             // the launch is sized for the whole batch, workgroups past it return
  double* res;          // [B][8][res_lanes(N)]: xf, xX, z[3], y[3] of every lane
  double* res_rho;      // [B]
  double* res_key;      // [B][2]: the primal / dual residual over its tolerance half way through the
                        // slice, then (at suspension) [b][0] = the iterations left, extrapolated from
                        // their decay since -- the resumed launch's order
  int32_t* res_i;       // [B][8]: next iteration, to the next check, to the next adaptation, rho
                        // updates, the half-way sample's iteration, 3 spare
};
constexpr int32_t kStatusSuspended = 100;  // (internal: the host loop resumes these)
constexpr int64_t res_lanes(int N) { return 16 * (int64_t)((N + 3) & ~3); }

// Doubles of engine workspace per instance: 0 up to 32 stages (everything in LDS);
// beyond, a 288-double pad, S^{-1} (N x 144 + 2), F W (N x 72), R^{-1} Q (N x 36),
// a zero block (72), beyond 49 stages the scaled constraint values (126 N - 18,
// rounded up to even), beyond 48 every lane's row of F_k (12 x 16 x the stage rows, N
// rounded up to 4); the F W block stays reserved (F W lives in LDS since round 3)
// (-DMPCQ_OCC16=3/4, an experiment: the 16-stage kernel in the beyond-32 layout, its
// scaled constraint values in the workspace too -- mpcq_engine.hip kOcc)
#if defined(MPCQ_OCC3) && !defined(MPCQ_OCC16)
#define MPCQ_OCC16 3
#elif defined(MPCQ_OCC4) && !defined(MPCQ_OCC16)
#define MPCQ_OCC16 4
#endif
#ifdef MPCQ_OCC16
constexpr bool work_occ16(int N) { return N == 16 && MPCQ_OCC16 > 2; }
#else
constexpr bool work_occ16(int) { return false; }
#endif
// The nested-dissection state solve (mpcq_engine.hip kND, round 6; an opt-in variant: measured
// slower than the two-ended sweep): at these horizons the scaled
// constraint values live in the workspace (72-double zero block + 126 N - 18, rounded up to
// even), which frees the LDS for the separator's spikes.  -DMPCQ_ND: N = 32; -DMPCQ_ND16: N = 16
// and 32.  Without either (the production build) the round-5 two-ended sweep at every horizon.
#if defined(MPCQ_ND16)
constexpr bool nd_layout(int N) { return N == 32 || N == 16; }
#elif defined(MPCQ_ND)
constexpr bool nd_layout(int N) { return N == 32; }
#else
constexpr bool nd_layout(int) { return false; }
#endif
constexpr int64_t work_doubles(int N) {
  if (nd_layout(N)) return 72 + ((126 * (int64_t)N - 18 + 1) & ~1);
  return (N > 32 || work_occ16(N)) ? 288 + (int64_t)N * (144 + 72 + 36) + 2 + 72 + ((N > 49 || work_occ16(N)) ? ((126 * N - 18 + 1) & ~1) : 0) +
                      (N > 48 ? (int64_t)12 * 16 * ((N + 3) & ~3) : 0)
                : 0;
}

// Planner launch (mpcq_planner.hip); layouts in include/mpcq.h (mpcq_plan_batch).
struct PlanArgs {
  int64_t batch;
  int N;
  unsigned ops;        // MPCQ_PLAN_* bits
  int k;
  const double* state; // [B][12]
  const double* v_cur; // [B][6] or null (state[6:12])
  const double* h;     // [B] or null (state[2])
  const double* l_feet;// [B][3][4]
  const double* v_ref; // [B][6]
  const int32_t* reduced; // [B] or null
  double* gait;        // [B][20][5] in/out
  int32_t* rot_flag;   // [B] in/out
  double* h_rot;       // [B] in/out
  double* xref;        // [B][12][N+1] in/out
  double* fsteps;      // [B][20][13] out
  int32_t* status;     // [B] or null
};

hipError_t launch_plan(const mpcq_planner_params& pp, const PlanArgs& a, hipStream_t s);

// Session epilogue (mpcq_session.hip): one robot per wave64.
struct SessionArgs {
  int64_t batch;
  const double* x;       // [B][24N] solution of this tick
  const double* xref;    // [B][12][N+1]
  const double* fsteps;  // [B][20][13]
  const double* gait;    // [B][20][5]
  int32_t* status;       // [B] engine status, overridden by a planner failure
  const int32_t* plan_status;  // [B]
  double* x_robot;       // [B][12][N]
  double* warm_x;        // [B][24N] next tick's warm start
  double* y;             // [B][44N] reset to 0 after a failed solve
  double* rho;           // [B]      reset to rho0 after a failed solve
  double rho0;
  double* cost;          // [B][13]
  double* q_w;           // [B][6]
  double* next_state;    // [B][12]
  double* next_l_feet;   // [B][3][4]
  double state_weights[12];
  double force_weight;
  double shoulders[8];
};

hipError_t launch_retrieve(int N, const SessionArgs& a, hipStream_t s);
// Dispatch order of the next tick's solve (mpcq_session.hip): the robots sorted by
// this tick's iteration counts, longest first (buckets of 16 iterations).
hipError_t launch_order(const int32_t* iters, int64_t batch, int32_t* order, hipStream_t s);

// Dispatch order of a batch solve by gait class (mpcq_order.hip, MPCQ_FLAG_ORDER_BY_CLASS):
// cls[B] = each instance's class slot, order[B] = the instances by the expected cost their
// class has shown on this context (sum / cnt: class_table_slots() entries), the most
// expensive first, index order inside a cost bucket; launch_class_learn adds a launch's
// iteration counts to the table.
int class_table_slots();
hipError_t launch_class_order(const double* fsteps, int64_t batch, int32_t* cls, const uint64_t* sum,
                              const uint32_t* cnt, int32_t* order, hipStream_t s);
hipError_t launch_class_learn(const int32_t* cls, const int32_t* iters, int64_t batch, uint64_t* sum,
                              uint32_t* cnt, hipStream_t s);
// Sliced solves: list[*count] = the instances of prev[0..n) (null: 0..n-1) whose status is
// kStatusSuspended, the largest key (key[2 id]: the iterations left, extrapolated) first, in
// prev's order inside a key bucket (one workgroup; buckets of 1/8 octave).
hipError_t launch_suspended(const int32_t* prev, int64_t n, const int32_t* status, const double* key,
                            int32_t* list, int32_t* count, hipStream_t s);

// Launchers (mpcq_engine.hip).  Return hipError_t.
hipError_t launch_formulate(int N, const mpcq_params& p, const LaunchArgs& a, hipStream_t s);
hipError_t launch_solve(int N, bool fused, const mpcq_params& p, const LaunchArgs& a, hipStream_t s);
// the horizons the engine is compiled for (mpcq_dispatch.cpp, Makefile)
#define MPCQ_HORIZONS(X)                                                                                     \
  X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22)  \
  X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32) X(33) X(34) X(35) X(36) X(37) X(38) X(39) X(40)  \
  X(41) X(42) X(43) X(44) X(45) X(46) X(47) X(48) X(49) X(50) X(51) X(52) X(53) X(54) X(55) X(56) X(57) X(58)  \
  X(59) X(60) X(61) X(62) X(63) X(64)
bool horizon_supported(int N);
int supported_horizons(int32_t* out, int cap);

}  // namespace mpcq
