/*
 * planner_oracle.c — CPU restatement of the reference FootstepPlanner (the
 * producer of MPC.run's xref / fsteps).  TEST INFRASTRUCTURE ONLY: used by
 * tests/ as the checker of mpcq_plan_batch; the product never links it.
 *
 * Restates, one instance at a time, in the reference's operation order
 * (numpy's rounding order: sequential cumsum, no fused multiply-adds except
 * inside np.dot, which BLAS computes with them):
 *   roll               FootstepPlanner.py:401-425
 *   compute_footsteps  FootstepPlanner.py:284-361
 *   compute_next_footstep (called as (v_ref, v_ref, h), FootstepPlanner.py:316)
 *                      FootstepPlanner.py:363-399
 *   getRefStates       FootstepPlanner.py:76-159 (rows it leaves alone keep
 *                      their previous values: xref is in/out)
 * Pinned by tests/golden/planner_golden.npz, captured from the unmodified
 * reference FootstepPlanner.py (tests/golden/gen_planner_golden.py): gait,
 * fsteps, xref and the state machine match it bit for bit on every tick.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/mpcq.h"

void oracle_default_planner_params(mpcq_planner_params* pp) {
  memset(pp, 0, sizeof(*pp));
  pp->dt = 0.02;
  pp->T_gait = 0.32;        /* FootstepPlanner.py:51 */
  pp->h_ref = 0.2027682;    /* processing.py:131 */
  pp->k_feedback = 0.03;    /* FootstepPlanner.py:20 */
  pp->L = 0.12;             /* FootstepPlanner.py:33 */
  pp->g = 9.81;             /* FootstepPlanner.py:30 */
  pp->t_stance = 0.16;      /* FootstepPlanner.py:376 */
  pp->cmd_threshold = 0.05; /* FootstepPlanner.py:130 */
  const double sh[8] = {0.19, 0.19, -0.19, -0.19, 0.15005, -0.15005, 0.15005, -0.15005};
  memcpy(pp->shoulders, sh, sizeof(sh)); /* FootstepPlanner.py:23-24 */
  const double ro[8] = {0.14, 0.14, -0.14, -0.14, 0.12, -0.12, 0.12, -0.12};
  memcpy(pp->reduced_offset, ro, sizeof(ro)); /* FootstepPlanner.py:320-322 */
}

/* numpy.linspace(a, b, n)[i] (endpoint): i * ((b - a) / (n - 1)) + a, last = b */
static double linspace_at(double a, double b, int n, int i) {
  if (n == 1) return a;
  if (i == n - 1) return b;
  const double step = (b - a) / (double)(n - 1);
  return (double)i * step + a;
}

/* roll (FootstepPlanner.py:401-425); returns 0 or MPCQ_STATUS_BAD_GAIT */
static int roll(double* gait) {
  int index = -1;
  for (int i = 0; i < 20; ++i)
    if (gait[5 * i] == 0.0) { index = i; break; }
  if (index < 0) return MPCQ_STATUS_BAD_GAIT; /* next(..., 0.0)[0] raises */
  const int last = (index + 19) % 20;           /* gait[index - 1], Python wraps -1 */
  int same = 1;
  for (int q = 1; q < 5; ++q)
    if (!(gait[q] == gait[5 * last + q])) same = 0;
  if (same) {
    gait[5 * last] += 1.0;
  } else {
    for (int q = 1; q < 5; ++q) gait[5 * index + q] = gait[q];
    gait[5 * index] = 1.0;
  }
  if (gait[0] > 1.0) {
    gait[0] -= 1.0;
  } else {
    double tmp[100];
    memcpy(tmp, gait + 5, 95 * sizeof(double));
    memcpy(gait, tmp, 95 * sizeof(double));
    for (int q = 0; q < 5; ++q) gait[95 + q] = 0.0;
  }
  return 0;
}

/* compute_next_footstep(v_cur = v_ref, v_ref, h) (FootstepPlanner.py:363-399), nf row-major 3x4 */
static void next_footstep(const mpcq_planner_params* pp, const double* v_ref, double h, double nf[12]) {
  const double* vc = v_ref; /* FootstepPlanner.py:316 passes v_ref twice */
  for (int e = 0; e < 12; ++e) nf[e] = 0.0;
  const double half = pp->t_stance * 0.5;
  for (int r = 0; r < 2; ++r)
    for (int q = 0; q < 4; ++q) nf[4 * r + q] += half * vc[r];
  for (int r = 0; r < 2; ++r)
    for (int q = 0; q < 4; ++q) nf[4 * r + q] += pp->k_feedback * (vc[r] - v_ref[r]);
  /* np.cross(v_cur[0:3], v_ref[3:6]) */
  double cr[2];
  {
    double t0 = vc[1] * v_ref[5];
    double t1 = vc[2] * v_ref[4];
    cr[0] = t0 - t1;
    t0 = vc[2] * v_ref[3];
    t1 = vc[0] * v_ref[5];
    cr[1] = t0 - t1;
  }
  const double coef = 0.5 * sqrt(h / pp->g);
  for (int r = 0; r < 2; ++r)
    for (int q = 0; q < 4; ++q) nf[4 * r + q] += coef * cr[r];
  for (int e = 0; e < 8; ++e) {
    if (nf[e] > pp->L) nf[e] = pp->L;
  }
  for (int e = 0; e < 8; ++e) {
    if (nf[e] < -pp->L) nf[e] = -pp->L;
  }
  for (int e = 0; e < 8; ++e) nf[e] += pp->shoulders[e];
}

/* compute_footsteps (FootstepPlanner.py:284-361); fsteps 20x13 row-major */
static int compute_footsteps(const mpcq_planner_params* pp, const double* gait, const double* l_feet,
                             const double* v_cur, const double* v_ref, double h, int reduced,
                             double* fsteps) {
  double fs[260];
  int rpt[20][12];
  for (int i = 0; i < 20; ++i) {
    fs[13 * i] = gait[5 * i];
    for (int c = 0; c < 12; ++c) {
      fs[13 * i + 1 + c] = NAN;
      rpt[i][c] = gait[5 * i + 1 + c / 3] == 1.0;
    }
  }
  for (int c = 0; c < 12; ++c) /* l_feet.ravel('F')[c] = l_feet[c % 3][c / 3] */
    if (rpt[0][c]) fs[1 + c] = l_feet[4 * (c % 3) + c / 3];
  double dt_cum = 0.0;
  int i = 1;
  for (;;) {
    if (i >= 20) return MPCQ_STATUS_BAD_GAIT; /* self.gait[20, 0]: IndexError */
    if (!(gait[5 * i] != 0.0)) break;
    dt_cum += gait[5 * (i - 1)] * pp->dt;
    for (int c = 0; c < 12; ++c)
      if (rpt[i - 1][c] && rpt[i][c]) fs[13 * i + 1 + c] = fs[13 * (i - 1) + 1 + c];
    int any = 0;
    for (int c = 0; c < 12; ++c) any |= (!rpt[i - 1][c]) && rpt[i][c];
    if (any) {
      double nf[12];
      next_footstep(pp, v_ref, h, nf);
      if (reduced)
        for (int e = 0; e < 8; ++e) nf[e] -= pp->reduced_offset[e];
      const double angle = v_ref[5] * dt_cum;
      const double co = cos(angle), si = sin(angle);
      const double R[9] = {co, -si, 0.0, si, co, 0.0, 0.0, 0.0, 1.0};
      double dx, dy;
      if (v_ref[5] != 0.0) {
        const double a = v_ref[5] * dt_cum;
        dx = (v_cur[0] * sin(a) + v_cur[1] * (cos(a) - 1.0)) / v_ref[5];
        dy = (v_cur[1] * sin(a) - v_cur[0] * (cos(a) - 1.0)) / v_ref[5];
      } else {
        dx = v_cur[0] * dt_cum;
        dy = v_cur[1] * dt_cum;
      }
      const double d[3] = {dx, dy, 0.0};
      for (int c = 0; c < 12; ++c) {
        if (!((!rpt[i - 1][c]) && rpt[i][c])) continue;
        const int q = c / 3, r = c % 3;
        /* (R @ nf)[r, q] + d[r]: numpy's dot goes through BLAS dgemm, which
           accumulates the 3 products left to right with fused multiply-adds
           (bit-identical to np.dot on the golden inputs; plain mul+add is not) */
        double v = R[3 * r] * nf[q];
        v = fma(R[3 * r + 1], nf[4 + q], v);
        v = fma(R[3 * r + 2], nf[8 + q], v);
        fs[13 * i + 1 + c] = v + d[r];
      }
    }
    ++i;
  }
  memcpy(fsteps, fs, sizeof(fs));
  return 0;
}

/* getRefStates (FootstepPlanner.py:76-159); xref 12x(N+1) row-major, in/out */
static void ref_states(const mpcq_planner_params* pp, int N, int k, const double* st,
                       const double* v_ref, int32_t* flag, double* h_rot, double* xref) {
  const int NP = N + 1;
  double* X = xref;
#define XR(r, j) X[(r) * NP + (j)]
  const double Tg = pp->T_gait, dt = pp->dt;
  for (int j = 1; j <= N; ++j) {
    const double yaw = linspace_at(0.0, Tg - dt, N, j - 1) * v_ref[5];
    const double c = cos(yaw), s = sin(yaw);
    XR(6, j) = v_ref[0] * c - v_ref[1] * s;
    XR(7, j) = v_ref[0] * s + v_ref[1] * c;
  }
  double a0 = 0.0, a1 = 0.0;
  for (int j = 1; j <= N; ++j) { /* dt * cumsum, then += lC */
    a0 += XR(6, j);
    a1 += XR(7, j);
    XR(0, j) = dt * a0 + st[0];
    XR(1, j) = dt * a1 + st[1];
  }
  if (k == 0)
    for (int j = 1; j <= N; ++j) XR(2, j) = pp->h_ref;
  for (int j = 1; j <= N; ++j) {
    XR(5, j) = v_ref[5] * linspace_at(dt, Tg, N, j - 1);
    XR(11, j) = v_ref[5];
  }
  for (int r = 0; r < 12; ++r) XR(r, 0) = st[r];
  const double step = pp->cmd_threshold;
  if (fabs(v_ref[2]) > step && *flag != 1) *flag = 1;
  if (fabs(v_ref[2]) > step && *flag == 1) {
    *h_rot += v_ref[2] * dt;
    for (int j = 1; j <= N; ++j) { XR(2, j) = *h_rot; XR(8, j) = v_ref[2]; }
    *flag = 1;
  } else if (fabs(v_ref[2]) < step && *flag == 1) {
    for (int j = 1; j <= N; ++j) { XR(8, j) = 0.0; XR(9, j) = 0.0; XR(10, j) = 0.0; }
    *flag = 2;
  } else if (*flag == 0) {
    for (int j = 1; j <= N; ++j) { XR(2, j) = pp->h_ref; XR(8, j) = 0.0; }
  }
  if (*flag != 0) {
    for (int j = 1; j <= N; ++j) {
      const double to = linspace_at(0.0, Tg - dt, N, j - 1);
      XR(3, j) = XR(3, 0) + v_ref[3] * to;
      XR(4, j) = XR(4, 0) + v_ref[4] * to;
      XR(9, j) = v_ref[3];
      XR(10, j) = v_ref[4];
    }
  }
#undef XR
}

/* One instance of mpcq_plan_batch.  Buffers change only when status == 0. */
int oracle_plan(const mpcq_planner_params* pp, int N, unsigned ops, int k, const double* state,
                const double* v_cur, const double* h, const double* l_feet, const double* v_ref,
                int reduced, double* gait, int32_t* rot_flag, double* h_rot, double* xref,
                double* fsteps) {
  double g[100];
  memcpy(g, gait, sizeof(g));
  if (ops & MPCQ_PLAN_ROLL) {
    const int st = roll(g);
    if (st) return st;
  }
  double fs[260];
  if (ops & MPCQ_PLAN_FOOTSTEPS) {
    const double* vc = v_cur ? v_cur : state + 6;
    const double hh = h ? *h : state[2];
    const int st = compute_footsteps(pp, g, l_feet, vc, v_ref, hh, reduced, fs);
    if (st) return st;
  }
  memcpy(gait, g, sizeof(g));
  if (ops & MPCQ_PLAN_FOOTSTEPS) memcpy(fsteps, fs, sizeof(fs));
  if (ops & MPCQ_PLAN_REFSTATES) ref_states(pp, N, k, state, v_ref, rot_flag, h_rot, xref);
  return 0;
}
