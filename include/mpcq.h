/*
 * mpcq.h — C ABI of the MI355X-native batched convex-MPC QP engine (libmpcq.so).
 *
 * Drop-in boundary for the hot path of thomascbrs/mpc-tsid: the QP formulation
 * in MPC.py and its OSQP solve.  Every entry point below names the reference
 * interface it replaces (file:line in the reference tree).  Plain C types only:
 * pointers + sizes, no torch / HIP types in the signatures.
 *
 * Problem (per instance, horizon N, MPC.py:98-288):
 *   x = [X_1..X_N (12 each), f_0..f_{N-1} (12 each)]     n = 24N variables
 *   rows: 12N dynamics | 12N swing mask | 20N friction    m = 44N constraints
 *   min 1/2 x'Px   s.t.  l <= A x <= u     (P diagonal, q = 0)
 * A is CSC with the fixed sparsity pattern of MPC.create_ML (nnz = 126N-18).
 *
 * Layouts (all C-order / row-major, float64):
 *   xref    [B][12][N+1]   column 0 = current state (MPC.py:466-467)
 *   fsteps  [B][20][13]    col 0 = phase duration, then foot xyz (NaN = swing)
 *   Ax      [B][nnz]       CSC data, pattern from mpcq_pattern()
 *   l, u    [B][m]
 *   x       [B][n], y [B][m], f0 [B][12]
 *
 * Conventions: functions return 0 on success, a negative MPCQ_E* code on an
 * API error (message via mpcq_last_error()).  Per-instance outcomes are
 * reported through the status array (OSQP codes, see MPCQ_STATUS_*).
 * Inputs are never mutated.  Calls are blocking unless MPCQ_FLAG_ASYNC.
 */
#ifndef MPCQ_H
#define MPCQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI changelog:
 *   2: eps_prim_inf / eps_dual_inf, dual_warm, infeasibility statuses
 *   3: info[b][3] = the ADMM's own exit status (before polish; was always 0),
 *      MPCQ_SV_ORDER added (MPCQ_SV_COUNT 16 -> 17), initialised to the identity */
#define MPCQ_ABI_VERSION 3

/* error codes (return values) */
#define MPCQ_OK 0
#define MPCQ_E_INVALID (-1)   /* bad argument */
#define MPCQ_E_DEVICE (-2)    /* HIP runtime error */
#define MPCQ_E_NOMEM (-3)     /* allocation failed */
#define MPCQ_E_UNSUPPORTED (-4) /* horizon N not compiled in */

/* per-instance status (OSQP 0.6 status values, plus formulation errors) */
#define MPCQ_STATUS_SOLVED 1
#define MPCQ_STATUS_SOLVED_INACCURATE 2
#define MPCQ_STATUS_PRIMAL_INFEASIBLE_INACCURATE 3
#define MPCQ_STATUS_DUAL_INFEASIBLE_INACCURATE 4
#define MPCQ_STATUS_MAX_ITER_REACHED (-2)
#define MPCQ_STATUS_PRIMAL_INFEASIBLE (-3)  /* OSQP 0.6 is_primal_infeasible: x, y, f0 are NaN */
#define MPCQ_STATUS_DUAL_INFEASIBLE (-4)    /* OSQP 0.6 is_dual_infeasible: x, y, f0 are NaN */
#define MPCQ_STATUS_NONFINITE (-10)      /* NaN/Inf reached the solver */
#define MPCQ_STATUS_BAD_GAIT (-11)       /* fsteps durations: no terminator / sum != N / NaN */
#define MPCQ_STATUS_FACTOR_FAILED (-12)  /* KKT block lost positive definiteness */
#define MPCQ_STATUS_BAD_BOUNDS (-13)     /* some l > u: osqp's setup / update reject the data
                                            (the python wrapper raises ValueError); no solve */

/* flags */
#define MPCQ_FLAG_DEVICE_PTRS 1u  /* every array argument is a device pointer on ctx's device */
#define MPCQ_FLAG_ASYNC 2u        /* do not synchronise the stream before returning (device ptrs only) */
/* mpcq_solve_batch only: dispatch the instances in the order of the mean iteration count
 * their gait class (the set of contact masks of their fsteps phases) has shown in this
 * context's earlier launches with this flag, the most expensive first (index order inside
 * a class and before any launch); the launch then adds its own counts.  Scheduling only:
 * every result is bit-identical with and without it.  No reference counterpart (the
 * reference solves one QP per tick). */
#define MPCQ_FLAG_ORDER_BY_CLASS 4u

/* formulation mode (MPC.py:491-494) */
#define MPCQ_MODE_UPDATE 0  /* k > 0: update_ML/update_NK with fsteps footholds */
#define MPCQ_MODE_SETUP 1   /* k == 0: create_ML/create_NK with the default footholds */

/*
 * Parameters.  mpcq_default_params() fills the reference constants:
 * dt 0.02, mass 2.50000279 (MPC.py:28), inertia gI (MPC.py:35-37), mu 0.9
 * (MPC.py:39), fz_max 25 (MPC.py:228), g 9.81 (MPC.py:201), state weights
 * (MPC.py:255-266), force weight 1e-5 (MPC.py:273-275), default footholds
 * (MPC.py:67-70) and the OSQP 0.6 settings used by MPC.py:414-416
 * (eps_abs = eps_rel = 1e-7, every other setting at the library default).
 */
typedef struct mpcq_params {
  /* --- formulation --- */
  double dt;
  double mass;
  double gI[9];             /* row-major 3x3 body inertia */
  double mu;
  double fz_max;
  double gravity;
  double state_weights[12]; /* P diagonal for [pos, rpy, linvel, angvel] */
  double force_weight;      /* P diagonal for every force component */
  double footholds[12];     /* default footholds, row-major 3x4 (setup mode) */
  /* --- OSQP settings --- */
  double rho;               /* 0.1 */
  double sigma;             /* 1e-6 */
  double alpha;             /* 1.6 */
  double eps_abs;           /* 1e-7 */
  double eps_rel;           /* 1e-7 */
  double adaptive_rho_tolerance; /* 5 */
  double delta;             /* polish regularisation 1e-6 */
  double eps_prim_inf;      /* 1e-4: primal infeasibility tolerance (OSQP 0.6 default) */
  double eps_dual_inf;      /* 1e-4: dual infeasibility tolerance (OSQP 0.6 default) */
  int32_t max_iter;         /* 4000 */
  int32_t check_termination;/* 25 */
  int32_t adaptive_rho;     /* 1 */
  int32_t adaptive_rho_interval; /* 100 = OSQP's non-timed rule (4 x check_termination) */
  int32_t scaling;          /* 10 Ruiz iterations */
  int32_t polish;           /* 0 off (OSQP default); 1 after SOLVED (OSQP); 2 also after
                               SOLVED_INACCURATE / MAX_ITER (status upgraded if it then meets eps) */
  int32_t polish_refine_iter; /* 3 */
  int32_t polish_rounds;    /* 1 = OSQP's single active-set guess; >1 iterates the
                               guess (primal-dual active set) until it repeats */
  int32_t dual_warm;        /* how warm_y / y are read and written (MPC.py:419-420):
                               0: osqp's unscaled duals (warm_start(y=) in, results.y out);
                               1: the solver's scaled workspace y, carried as is across the
                                  re-scaled update(Ax=) + warm_start(x=) of the next tick --
                                  what osqp 0.6 does between the reference's ticks */
  int32_t reserved[7];
} mpcq_params;

typedef struct mpcq_ctx mpcq_ctx;

/* ---- metadata / pattern -------------------------------------------------- */
int mpcq_abi_version(void);
void mpcq_default_params(mpcq_params* p);
/* Dimensions for horizon N: n = 24N, m = 44N, nnz = 126N - 18. */
int mpcq_dims(int n_steps, int32_t* n, int32_t* m, int32_t* nnz);
/* CSC pattern of MPC.create_ML (MPC.py:98-151): indptr[n+1], indices[nnz]. */
int mpcq_pattern(int n_steps, int32_t* indptr, int32_t* indices);
/* Horizons compiled into the HIP engine (writes up to cap values). */
int mpcq_supported_horizons(int32_t* out, int cap);
const char* mpcq_last_error(void);
/* Build stamp of this library (no reference counterpart: provenance for profiles):
 * "src_sha256=<16 hex> arch=gfx950", the hex the first 16 of sha256 over the csrc .hip files,
 * the assembly pass, the Makefile, the headers, the .cpp units and the effective compiler
 * flags (csrc/stamp.py); the stamps build appends "+stamps", an experiment variant
 * "+exp:<name>:<hash>" (tools/build_variant.sh).  bench.py drops a committed PMC figure
 * whose stamp differs from the running library's. */
const char* mpcq_build_info(void);

/* ---- context --------------------------------------------------------------
 * Replaces MPC.MPC(dt, n_steps, T_gait) (MPC.py:22-82) + osqp.OSQP() (MPC.py:73).
 * One context per (device, host thread).  The context owns device scratch. */
int mpcq_create(int device, int n_steps, const mpcq_params* params, mpcq_ctx** out);
int mpcq_destroy(mpcq_ctx* ctx);
/* HIP stream (hipStream_t passed as void*) for subsequent launches; NULL = ctx's own stream. */
int mpcq_set_stream(mpcq_ctx* ctx, void* stream);
/* Device time of the last launch of each kernel (ms, hipEvent timing on ctx's stream; a
 * sliced solve: from its first slice's start to its last slice's end). */
int mpcq_last_kernel_ms(mpcq_ctx* ctx, double* formulate_ms, double* solve_ms);
/* Sliced batch solves (no reference counterpart: a dispatch policy, no result changes).
 * slice_iters > 0: beyond 16 stages, the batch solves of this context (mpcq_solve_batch,
 * mpcq_qp_solve_batch) run as two launches: the first suspends every instance still iterating
 * at the first ADMM segment end (check / adaptive-rho / max_iter boundary) after slice_iters
 * iterations and saves its iterate in device scratch; the second resumes the suspended ones
 * (formulation, scaling and the factorisation at the saved rho recomputed), the farthest from
 * convergence (the iterations left, extrapolated from the residuals' decay) first, to their
 * end.  Every output is bit-identical to the unsliced solve's; long instances no longer hold a CU slot
 * past the others and start first once known, so a batch whose instances fill the CUs in
 * several rounds ends sooner.  No host synchronisation: the second
 * launch reads its workgroup count on the device (MPCQ_FLAG_ASYNC holds).  0 (the default), a
 * slice of max_iter or more, and horizons up to 16: one launch. */
int mpcq_set_slice(mpcq_ctx* ctx, int32_t slice_iters);

/* ---- formulation -----------------------------------------------------------
 * Replaces MPC.construct_gait + update_matrices (MPC.py:635-652, 290-378) in
 * MODE_UPDATE, and construct_gait + create_matrices (MPC.py:84-234) in
 * MODE_SETUP: writes A.data (CSC order), l and u for each instance.
 * status[b] = 0 or MPCQ_STATUS_BAD_GAIT. */
int mpcq_formulate_batch(mpcq_ctx* ctx, int64_t batch, const double* xref,
                         const double* fsteps, int mode, double* Ax, double* l,
                         double* u, int32_t* status, uint32_t flags);

/* ---- QP solve --------------------------------------------------------------
 * Replaces osqp.OSQP.update(Ax=, l=, u=) + warm_start(x=) + solve()
 * (MPC.py:419-428; osqp 0.6 ADMM).  P, q come from params (constant).
 * warm_x [B][n], warm_y [B][m], rho_in [B] are optional (NULL = cold start,
 * rho = params.rho).  x, y, rho_out, iters optional outputs (NULL = skip).
 * info [B][4] (optional): rho updates (refactorisations after the first),
 * polish result (0 not run, 1 accepted, -1 rejected), polish rounds run, and
 * the ADMM's own exit status before polish (with polish = 2 a MAX_ITER /
 * SOLVED_INACCURATE exit that polish upgrades reports SOLVED in status and the
 * ADMM's code here). */
int mpcq_qp_solve_batch(mpcq_ctx* ctx, int64_t batch, const double* Ax,
                        const double* l, const double* u, const double* warm_x,
                        const double* warm_y, const double* rho_in, double* x,
                        double* y, int32_t* status, int32_t* iters,
                        double* rho_out, int32_t* info, uint32_t flags);

/* ---- fused hot path --------------------------------------------------------
 * Replaces MPC.run(k, xref, fsteps) (MPC.py:460-514) for a batch: formulation
 * + OSQP solve (with the osqp workspace carried between ticks: warm_x, warm_y,
 * rho_in, as mpcq_qp_solve_batch) + retrieve_result (MPC.py:432-458) in one
 * launch.  f0 [B][12] = f_applied; x [B][n], y [B][m], rho_out [B] optional. */
int mpcq_solve_batch(mpcq_ctx* ctx, int64_t batch, const double* xref,
                     const double* fsteps, int mode, const double* warm_x,
                     const double* warm_y, const double* rho_in, double* f0, double* x,
                     double* y, double* rho_out, int32_t* status, int32_t* iters,
                     int32_t* info, uint32_t flags);

/* ---- footstep planner ------------------------------------------------------
 * The producer of (xref, fsteps): FootstepPlanner.py.  Per instance the
 * planner keeps the reference object's mutable state — the gait table
 * gait [20][5] (durations + contact bits, FootstepPlanner.py:58-62,193-213),
 * the rotation-command state machine (flag_rotation_command,
 * h_rotation_command, FootstepPlanner.py:67-68,130-154) and xref itself
 * (getRefStates only rewrites some rows in some states, so xref is in/out).
 *
 * Parameters (mpcq_default_planner_params): FootstepPlanner.py:18-52,321,352. */
typedef struct mpcq_planner_params {
  double dt;            /* MPC time step, 0.02 */
  double T_gait;        /* 0.32 (FootstepPlanner.py:51); getRefStates' linspace end points */
  double h_ref;         /* 0.2027682 (processing.py:131 passes it to getRefStates) */
  double k_feedback;    /* 0.03 */
  double L;             /* 0.12: bound on the (x, y) deviation from the shoulders */
  double g;             /* 9.81 */
  double t_stance;      /* 0.16 (compute_next_footstep) */
  double cmd_threshold; /* 0.05: joystick dead band of the height command */
  double shoulders[8];  /* row-major 2x4: x of FL FR HL HR, then y */
  double reduced_offset[8]; /* row-major 2x4 subtracted when reduced (FootstepPlanner.py:320-322) */
  int32_t reserved[8];
} mpcq_planner_params;

/* operations of mpcq_plan_batch, applied in this order */
#define MPCQ_PLAN_ROLL 1u       /* FootstepPlanner.roll (FootstepPlanner.py:401-425) */
#define MPCQ_PLAN_FOOTSTEPS 2u  /* compute_footsteps (FootstepPlanner.py:284-361) */
#define MPCQ_PLAN_REFSTATES 4u  /* getRefStates (FootstepPlanner.py:76-159) */
/* update_fsteps(k > 0) + getRefStates: the once-per-tick sequence of processing.py:81-131 */
#define MPCQ_PLAN_TICK (MPCQ_PLAN_ROLL | MPCQ_PLAN_FOOTSTEPS | MPCQ_PLAN_REFSTATES)

void mpcq_default_planner_params(mpcq_planner_params* pp);

/*
 * Replaces FootstepPlanner.update_fsteps(k, l_feet, v_cur, v_ref, h, oMl, _, reduced)
 * (FootstepPlanner.py:427-459, minus its viewer code) and getRefStates(k, T_gait,
 * lC, abg, lV, lW, v_ref, h_ref) (FootstepPlanner.py:76-159) for a batch.
 *   ops       MPCQ_PLAN_* bits
 *   k         getRefStates' k (only k == 0 is distinguished, FootstepPlanner.py:105)
 *   state     [B][12] lC, abg, lV, lW (local frame)             REFSTATES
 *   v_cur     [B][6]  compute_footsteps' v_cur; NULL = state[6:12] (processing.py:81)
 *   h         [B]     compute_footsteps' h;    NULL = state[2]   (processing.py:82)
 *   l_feet    [B][3][4] feet positions, local frame                FOOTSTEPS
 *   v_ref     [B][6]
 *   reduced   [B] int32, NULL = 0
 *   gait      [B][20][5]  in/out
 *   rot_flag  [B] int32 in/out, h_rot [B] in/out   (REFSTATES; 0 / 0.2 initially)
 *   xref      [B][12][N+1] in/out                                  REFSTATES
 *   fsteps    [B][20][13] out                                      FOOTSTEPS
 *   status    [B] out (optional): 0, or MPCQ_STATUS_BAD_GAIT where the reference
 *             raises (gait table without a zero-duration terminator / empty); the
 *             instance's buffers are then left unchanged.  Otherwise the table
 *             is followed exactly as the reference indexes it (an empty first row
 *             makes roll() look at row -1 = row 19, as Python does). */
int mpcq_plan_batch(mpcq_ctx* ctx, const mpcq_planner_params* pp, int64_t batch, uint32_t ops,
                    int k, const double* state, const double* v_cur, const double* h,
                    const double* l_feet, const double* v_ref, const int32_t* reduced,
                    double* gait, int32_t* rot_flag, double* h_rot, double* xref, double* fsteps,
                    int32_t* status, uint32_t flags);

/* ---- closed-loop session ---------------------------------------------------
 * B robots, each running the reference's once-per-tick MPC sequence
 * (processing.py:81-131 + MPC.run, MPC.py:460-514) with every piece of state
 * the reference keeps between ticks resident in HBM:
 *   FootstepPlanner: gait table, rotation state machine, xref, fsteps;
 *   MPC / osqp workspace: x (the next tick's warm start is x shifted by one
 *   stage, MPC.py:403-406), y and rho (kept by osqp across solves), q_w.
 * A tick is three launches on the context's stream, no host round trip:
 *   planner (roll + compute_footsteps + getRefStates; at k == 0 the extra
 *   compute_footsteps of processing.py:80-82 first) -> fused formulation + OSQP
 *   solve (k == 0: create_matrices, cold start; k > 0: update_matrices, warm) ->
 *   retrieve (f_applied, x_robot, q_next / v_next, q_w, the Logger's cost
 *   components, the next warm start, the virtual robot's next state).
 *
 * Virtual robot (optional): passing state == NULL / l_feet == NULL to a tick
 * takes the robot's state from the previous tick's prediction x_robot[:, 0],
 * re-expressed in the new local frame (origin under the base, yaw removed,
 * Interface.py:100-138), and the stance feet from the previous fsteps — the
 * "MPC future state as the robot state" path of processing.py:33-38.  It makes
 * a closed loop run entirely on the device (tests, benchmarks). */
typedef struct mpcq_session mpcq_session;

/* gait0 [B][20][5] (NULL: create_walking_trot for this ctx's horizon, FootstepPlanner.py:193-214).
 * pp NULL = mpcq_default_planner_params.  The session keeps ctx (and its stream). */
int mpcq_session_create(mpcq_ctx* ctx, int64_t batch, const mpcq_planner_params* pp,
                        const double* gait0, mpcq_session** out);
int mpcq_session_destroy(mpcq_session* s);

/* One tick for every robot.  state [B][12] (lC, abg, lV, lW), l_feet [B][3][4],
 * v_ref [B][6], reduced [B] (NULL = 0); host pointers, or device pointers with
 * MPCQ_FLAG_DEVICE_PTRS.  state / l_feet NULL = the virtual robot (above).
 * k = MPC tick index (k == 0: first tick, MPC.py:491).  Blocking unless
 * MPCQ_FLAG_ASYNC together with MPCQ_FLAG_DEVICE_PTRS.
 * From the second tick on, the solve dispatches the robots longest-first by the
 * previous tick's iteration counts (a fourth, one-workgroup launch after the
 * retrieve builds the order); results do not depend on it.  The environment
 * variable MPCQ_DISPATCH_ORDER=0, read at mpcq_session_create, keeps index order
 * (timing comparisons only). */
int mpcq_session_tick(mpcq_session* s, int k, const double* state, const double* l_feet,
                      const double* v_ref, const int32_t* reduced, uint32_t flags);

/* Per-robot arrays a session holds (mpcq_session_read / mpcq_session_device_ptr). */
#define MPCQ_SV_F0 0        /* [B][12]     f_applied (MPC.py:441-444) */
#define MPCQ_SV_X 1         /* [B][24N]    QP solution x */
#define MPCQ_SV_X_ROBOT 2   /* [B][12][N]  x_robot = x states + xref[:, 1:] (MPC.py:437-449) */
#define MPCQ_SV_Q_W 3       /* [B][6]      world pose (MPC.py:503-510) */
#define MPCQ_SV_COST 4      /* [B][13]     Logger.log_cost_function (Logger.py:406-418) */
#define MPCQ_SV_XREF 5      /* [B][12][N+1] */
#define MPCQ_SV_FSTEPS 6    /* [B][20][13] */
#define MPCQ_SV_GAIT 7      /* [B][20][5] */
#define MPCQ_SV_STATUS 8    /* [B] int32: OSQP status, or MPCQ_STATUS_BAD_GAIT from the planner */
#define MPCQ_SV_ITERS 9     /* [B] int32 */
#define MPCQ_SV_RHO 10      /* [B] */
#define MPCQ_SV_Y 11        /* [B][44N] */
#define MPCQ_SV_STATE 12    /* [B][12]     the virtual robot's next state */
#define MPCQ_SV_L_FEET 13   /* [B][3][4]   the virtual robot's next feet */
#define MPCQ_SV_ROT_FLAG 14 /* [B] int32 */
#define MPCQ_SV_H_ROT 15    /* [B] */
#define MPCQ_SV_ORDER 16    /* [B] int32: the next tick's dispatch order (read-only: a permutation of
                               0..B-1, longest previous solve first, buckets of 16 iterations; the
                               identity until the first tick) */
#define MPCQ_SV_COUNT 17
/* Copy array `what` to dst (host, or device with MPCQ_FLAG_DEVICE_PTRS); blocking. */
int mpcq_session_read(mpcq_session* s, int what, void* dst, uint32_t flags);
/* Overwrite array `what` from src (host, or device with MPCQ_FLAG_DEVICE_PTRS); blocking.
 * MPCQ_SV_ORDER is read-only (MPCQ_E_INVALID). */
int mpcq_session_write(mpcq_session* s, int what, const void* src, uint32_t flags);
/* Device address of array `what` (valid until mpcq_session_destroy).  The engine reads
 * MPCQ_SV_ORDER as its workgroup -> robot map: writing through its device address is not
 * allowed (a non-permutation would solve some robots twice and others not at all). */
int mpcq_session_device_ptr(mpcq_session* s, int what, void** out);

/* ---- diagnostics -----------------------------------------------------------
 * Device buffer [B][16] (uint64) that a diagnostic build of the library
 * (compiled with -DMPCQ_STAMPS, libmpcq_stamps.so) fills with per-phase
 * s_memtime cycle counts of thread 0; ignored by the shipped build. */
int mpcq_debug_set_stamps(mpcq_ctx* ctx, void* device_buffer);

#ifdef __cplusplus
}
#endif
#endif /* MPCQ_H */
