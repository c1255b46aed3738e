/*
 * mpcq_oracle.c — CPU restatement of the reference hot path.  TEST
 * INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker.  The product (libmpcq.so) never
 * links, loads or calls this file.
 *
 * What it restates:
 *  1. MPC.py formulation (update and setup modes) — construct_gait
 *     (MPC.py:635-652), construct_S (MPC.py:611-633), create_ML / update_ML
 *     (MPC.py:98-190, 316-360), create_NK / update_NK (MPC.py:192-234,
 *     362-378), create_weight_matrices (MPC.py:236-288), utils.getSkew
 *     (utils.py:179-185).  Pinned against A.data / l / u captured from the
 *     unmodified reference (tests/golden/gen_golden.py).
 *  2. The OSQP 0.6 ADMM that MPC.py:413-428 calls (third-party, unpinned,
 *     absent from the reference tree and from this image).  Restated from the
 *     published algorithm (Stellato et al., "OSQP: an operator splitting solver
 *     for quadratic programs", Math. Prog. Comp. 2020) and the 0.6 defaults:
 *     Ruiz scaling (10 passes + cost scaling), rho 0.1, rho_eq = 1e3 rho,
 *     sigma 1e-6, alpha 1.6, termination check every 25 iterations with
 *     unscaled residuals, adaptive rho (interval = 4 x check_termination, the
 *     library's non-timed rule), max_iter 4000, optional polish (delta 1e-6,
 *     3 refinement steps), OSQP 0.6's infeasibility detection
 *     (auxil.c is_primal_infeasible / is_dual_infeasible on the last iteration's
 *     delta_y / delta_x at every termination check, eps_prim_inf = eps_dual_inf
 *     = 1e-4; statuses -3 / -4, and 3 / 4 from the approximate check at
 *     max_iter; x and y NaN then, as osqp's store_solution) -- every instance
 *     MPC.py builds is feasible (f = 0 with the dynamics roll-out satisfies all
 *     rows), so only hand-made data reach them.  params.dual_warm = 1 reads and
 *     writes y in the solver's scaled coordinates, the workspace y osqp carries
 *     across the reference's update(Ax=) + warm_start(x=) (MPC.py:419-420).
 *     The linear system is the reduced KKT P + sigma I + A' R A,
 *     factored as a block-tridiagonal Cholesky over stages z_k = [f_k; X_k+1]
 *     (exact, like OSQP's QDLDL on the quasi-definite form).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "../include/mpcq.h"

#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define RHO_TOL 1e-4
#define DIV_TOL 1e-30

/* ------------------------------------------------------------------------ */
/* parameters (MPC.py:25-39, 67-70, 201, 228, 255-275; MPC.py:414-416)       */
void oracle_default_params(mpcq_params* p) {
  memset(p, 0, sizeof(*p));
  p->dt = 0.02;
  p->mass = 2.50000279;
  const double gI[9] = {3.09249e-2, -8.00101e-7, 1.865287e-5,
                        -8.00101e-7, 5.106100e-2, 1.245813e-4,
                        1.865287e-5, 1.245813e-4, 6.939757e-2};
  memcpy(p->gI, gI, sizeof(gI));
  p->mu = 0.9;
  p->fz_max = 25.0;
  p->gravity = 9.81;
  const double w[12] = {0.1, 0.1, 1.0, 0.11, 0.11, 0.11, 2.0 * sqrt(0.1),
                        2.0 * sqrt(0.1), 2.0 * sqrt(1.0), 0.05 * sqrt(0.11),
                        0.05 * sqrt(0.11), 0.05 * sqrt(0.11)};
  memcpy(p->state_weights, w, sizeof(w));
  p->force_weight = 1.0e-5;
  const double fh[12] = {0.19, 0.19, -0.19, -0.19, 0.15005, -0.15005,
                         0.15005, -0.15005, 0.0, 0.0, 0.0, 0.0};
  memcpy(p->footholds, fh, sizeof(fh));
  p->rho = 0.1;
  p->sigma = 1e-6;
  p->alpha = 1.6;
  p->eps_abs = 1e-7;
  p->eps_rel = 1e-7;
  p->adaptive_rho_tolerance = 5.0;
  p->delta = 1e-6;
  p->eps_prim_inf = 1e-4;
  p->eps_dual_inf = 1e-4;
  p->max_iter = 4000;
  p->check_termination = 25;
  p->adaptive_rho = 1;
  p->adaptive_rho_interval = 100;
  p->scaling = 10;
  p->polish = 0;
  p->polish_refine_iter = 3;
  p->polish_rounds = 1;
  p->dual_warm = 0;
}

/* ------------------------------------------------------------------------ */
/* CSC pattern of create_ML (dense -> csc_matrix, MPC.py:103-151)            */
int oracle_dims(int N, int32_t* n, int32_t* m, int32_t* nnz) {
  if (N < 2) return -1;
  *n = 24 * N;
  *m = 44 * N;
  *nnz = 126 * N - 18;
  return 0;
}

int oracle_pattern(int N, int32_t* indptr, int32_t* indices) {
  int pos = 0;
  for (int c = 0; c < 12 * N; ++c) {
    int k = c / 12, i = c % 12;
    indptr[c] = pos;
    indices[pos++] = c; /* -I of dynamics row block k */
    if (k < N - 1) {    /* A of dynamics row block k+1 */
      if (i >= 6) indices[pos++] = 12 * (k + 1) + i - 6;
      indices[pos++] = 12 * (k + 1) + i;
    }
  }
  for (int k = 0; k < N; ++k)
    for (int j = 0; j < 4; ++j)
      for (int c = 0; c < 3; ++c) {
        int col = 12 * N + 12 * k + 3 * j + c;
        indptr[col] = pos;
        indices[pos++] = 12 * k + 6 + c;
        indices[pos++] = 12 * k + 9;
        indices[pos++] = 12 * k + 10;
        indices[pos++] = 12 * k + 11;
        indices[pos++] = 12 * N + 12 * k + 3 * j + c;
        int fr = 24 * N + 20 * k + 5 * j;
        if (c == 0) { indices[pos++] = fr + 0; indices[pos++] = fr + 1; }
        if (c == 1) { indices[pos++] = fr + 2; indices[pos++] = fr + 3; }
        if (c == 2) for (int t = 0; t < 5; ++t) indices[pos++] = fr + t;
      }
  indptr[24 * N] = pos;
  return pos;
}

/* ------------------------------------------------------------------------ */
/* formulation                                                               */
static void inv3(const double* M, double* R) {
  double a = M[0], b = M[1], c = M[2], d = M[3], e = M[4], f = M[5], g = M[6],
         h = M[7], i = M[8];
  double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
  double det = a * A + b * B + c * C;
  double id = 1.0 / det;
  R[0] = A * id; R[1] = -(b * i - c * h) * id; R[2] = (b * f - c * e) * id;
  R[3] = B * id; R[4] = (a * i - c * g) * id;  R[5] = -(a * f - c * d) * id;
  R[6] = C * id; R[7] = -(a * h - b * g) * id; R[8] = (a * e - b * d) * id;
}

/* B rows 9..11 for one stage: dt * inv(Rz(yaw) gI) * skew(lever_i)
 * (MPC.py:339-345 / 171-178). lever[3][4] column i = foot i. out[3][12]. */
static void stage_B(const mpcq_params* p, double yaw, const double lever[3][4],
                    double out[3][12]) {
  double c = cos(yaw), s = sin(yaw);
  double R[9] = {c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0};
  double M[9], Mi[9];
  for (int r = 0; r < 3; ++r)
    for (int t = 0; t < 3; ++t)
      M[3 * r + t] = R[3 * r + 0] * p->gI[0 * 3 + t] + R[3 * r + 1] * p->gI[1 * 3 + t] +
                     R[3 * r + 2] * p->gI[2 * 3 + t];
  inv3(M, Mi);
  for (int i = 0; i < 4; ++i) {
    double a0 = lever[0][i], a1 = lever[1][i], a2 = lever[2][i];
    double S[9] = {0.0, -a2, a1, a2, 0.0, -a0, -a1, a0, 0.0};
    for (int r = 0; r < 3; ++r)
      for (int cc = 0; cc < 3; ++cc)
        out[r][3 * i + cc] = p->dt * (Mi[3 * r + 0] * S[0 * 3 + cc] + Mi[3 * r + 1] * S[1 * 3 + cc] +
                                      Mi[3 * r + 2] * S[2 * 3 + cc]);
  }
}

/* construct_gait + phase walk: returns number of phases or -1 (bad gait). */
static int parse_gait(int N, const double* fsteps, int dur[20], int contact[20][4]) {
  int idx = -1;
  for (int j = 0; j < 20; ++j)
    if (fsteps[13 * j] == 0.0) { idx = j; break; }
  if (idx < 0) return -1; /* MPC.py:646 raises when no zero-duration row */
  int total = 0;
  for (int j = 0; j < idx; ++j) {
    double d = fsteps[13 * j];
    if (!(fabs(d) < 1e6)) return -1; /* NaN / inf: np.int() raises */
    int di = (int)d;                  /* np.int truncates toward zero */
    if (di < 0) return -1;
    dur[j] = di;
    total += di;
    for (int f = 0; f < 4; ++f) {
      double x = fsteps[13 * j + 1 + 3 * f];
      contact[j][f] = !(isnan(x) || x == 0.0);
    }
  }
  if (total != N) return -1; /* construct_S / update_ML need sum == N */
  return idx;
}

int oracle_formulate(const mpcq_params* p, int N, const double* xref, const double* fsteps,
                     int mode, double* Ax, double* l, double* u) {
  int dur[20], contact[20][4];
  int nph = parse_gait(N, fsteps, dur, contact);
  if (nph < 0) return MPCQ_STATUS_BAD_GAIT;
  const int NP1 = N + 1;
#define XR(r, k) xref[(r) * NP1 + (k)]
  /* constant part of the X columns */
  int pos = 0;
  for (int c = 0; c < 12 * N; ++c) {
    int k = c / 12, i = c % 12;
    Ax[pos++] = -1.0;
    if (k < N - 1) {
      if (i >= 6) Ax[pos++] = p->dt;
      Ax[pos++] = 1.0;
    }
  }
  const double dtm = p->dt / p->mass;
  int k = 0;
  for (int j = 0; j < nph; ++j) {
    for (int kk = 0; kk < dur[j]; ++kk, ++k) {
      double lever[3][4], B[3][12];
      for (int f = 0; f < 4; ++f)
        for (int r = 0; r < 3; ++r) {
          double ft;
          if (mode == MPCQ_MODE_SETUP) ft = p->footholds[4 * r + f];
          else {
            ft = fsteps[13 * j + 1 + 3 * f + r];
            if (isnan(ft)) ft = 0.0; /* MPC.py:327 */
          }
          lever[r][f] = ft - XR(r, k);
        }
      stage_B(p, XR(5, k), lever, B);
      for (int f = 0; f < 4; ++f)
        for (int c = 0; c < 3; ++c) {
          Ax[pos++] = dtm;
          Ax[pos++] = B[0][3 * f + c];
          Ax[pos++] = B[1][3 * f + c];
          Ax[pos++] = B[2][3 * f + c];
          Ax[pos++] = 1.0 - (double)contact[j][f]; /* S_gait (MPC.py:628) */
          if (c < 2) { Ax[pos++] = 1.0; Ax[pos++] = -1.0; }
          else for (int t = 0; t < 4; ++t) Ax[pos++] = -p->mu;
          if (c == 2) Ax[pos++] = -1.0;
        }
    }
  }
  /* bounds (MPC.py:197-232, 366-378, 410) */
  const double mg8 = -(-p->gravity * p->dt);
  for (int kb = 0; kb < N; ++kb)
    for (int r = 0; r < 12; ++r) {
      double v = (r == 8) ? mg8 : -0.0;
      if (kb == 0) {
        double ax0 = -XR(r, 0);
        if (r < 6) ax0 = ax0 + p->dt * (-XR(r + 6, 0));
        v = v + ax0;
      }
      double dv;
      if (kb >= 1) {
        dv = -XR(r, kb);
        if (r < 6) dv = dv + (-p->dt) * XR(r + 6, kb);
        dv = dv + XR(r, kb + 1);
      } else {
        dv = XR(r, 1);
      }
      v = v + dv;
      u[12 * kb + r] = v;
      l[12 * kb + r] = v;
    }
  for (int r = 12 * N; r < 24 * N; ++r) { u[r] = 0.0; l[r] = 0.0; }
  for (int r = 24 * N; r < 44 * N; ++r) {
    u[r] = 0.0;
    l[r] = ((r - 24 * N) % 5 == 4) ? -p->fz_max : -INFINITY;
  }
#undef XR
  return 0;
}

/* ------------------------------------------------------------------------ */
/* problem workspace                                                         */
typedef struct {
  int N, n, m, nnz;
  int32_t *colptr, *rowidx, *rowptr, *colidx, *cscpos;
  int32_t *stage, *loc;
  /* scaled data */
  double *Pd, *A, *lo, *hi, *D, *E, c;
  double *rho;
  /* block-tridiagonal factor */
  double *Kd, *Ko;
  /* ADMM vectors */
  double *x, *z, *y, *xt, *zt, *xp, *zp, *rhs, *w, *Ax, *Px, *Aty, *tmpn, *tmpm;
  double *dy, *dx, *tmpm2, *tmpn2;  /* delta_y, delta_x of the last iteration (osqp update_y / update_x) */
  int *ctype;
} Work;

static void* xalloc(size_t n) { void* p = calloc(n, 1); return p; }

static void work_free(Work* W) {
  void* ptrs[] = {W->colptr, W->rowidx, W->rowptr, W->colidx, W->cscpos, W->stage, W->loc,
                  W->Pd, W->A, W->lo, W->hi, W->D, W->E, W->rho, W->Kd, W->Ko,
                  W->x, W->z, W->y, W->xt, W->zt, W->xp, W->zp, W->rhs, W->w, W->Ax,
                  W->Px, W->Aty, W->tmpn, W->tmpm, W->ctype, W->dy, W->dx, W->tmpm2, W->tmpn2};
  for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i) free(ptrs[i]);
}

static int work_init(Work* W, int N) {
  memset(W, 0, sizeof(*W));
  W->N = N;
  oracle_dims(N, &W->n, &W->m, &W->nnz);
  int n = W->n, m = W->m, nnz = W->nnz;
  W->colptr = xalloc(sizeof(int32_t) * (n + 1));
  W->rowidx = xalloc(sizeof(int32_t) * nnz);
  W->rowptr = xalloc(sizeof(int32_t) * (m + 1));
  W->colidx = xalloc(sizeof(int32_t) * nnz);
  W->cscpos = xalloc(sizeof(int32_t) * nnz);
  W->stage = xalloc(sizeof(int32_t) * n);
  W->loc = xalloc(sizeof(int32_t) * n);
  W->Pd = xalloc(8 * n); W->A = xalloc(8 * nnz); W->lo = xalloc(8 * m); W->hi = xalloc(8 * m);
  W->D = xalloc(8 * n); W->E = xalloc(8 * m); W->rho = xalloc(8 * m);
  W->Kd = xalloc(8 * (size_t)N * 576); W->Ko = xalloc(8 * (size_t)N * 576);
  double** vn[] = {&W->x, &W->xt, &W->xp, &W->rhs, &W->Px, &W->Aty, &W->tmpn, &W->dx, &W->tmpn2};
  for (size_t i = 0; i < 9; ++i) *vn[i] = xalloc(8 * n);
  double** vm[] = {&W->z, &W->y, &W->zt, &W->zp, &W->w, &W->Ax, &W->tmpm, &W->dy, &W->tmpm2};
  for (size_t i = 0; i < 9; ++i) *vm[i] = xalloc(8 * m);
  W->ctype = xalloc(sizeof(int) * m);
  if (!W->ctype || !W->tmpm) return -1;
  oracle_pattern(N, W->colptr, W->rowidx);
  /* CSR view */
  int32_t* cnt = xalloc(sizeof(int32_t) * (m + 1));
  for (int p = 0; p < nnz; ++p) cnt[W->rowidx[p] + 1]++;
  for (int r = 0; r < m; ++r) cnt[r + 1] += cnt[r];
  memcpy(W->rowptr, cnt, sizeof(int32_t) * (m + 1));
  for (int c = 0; c < n; ++c)
    for (int p = W->colptr[c]; p < W->colptr[c + 1]; ++p) {
      int r = W->rowidx[p];
      int q = cnt[r]++;
      W->colidx[q] = c;
      W->cscpos[q] = p;
    }
  free(cnt);
  for (int c = 0; c < n; ++c) {
    if (c < 12 * N) { W->stage[c] = c / 12; W->loc[c] = 12 + c % 12; }
    else { W->stage[c] = (c - 12 * N) / 12; W->loc[c] = (c - 12 * N) % 12; }
  }
  return 0;
}

/* y = A x (scaled data) */
static void mat_vec(const Work* W, const double* x, double* y) {
  for (int r = 0; r < W->m; ++r) {
    double s = 0.0;
    for (int q = W->rowptr[r]; q < W->rowptr[r + 1]; ++q) s += W->A[W->cscpos[q]] * x[W->colidx[q]];
    y[r] = s;
  }
}
/* y = A' x */
static void mat_tvec(const Work* W, const double* x, double* y) {
  for (int c = 0; c < W->n; ++c) {
    double s = 0.0;
    for (int p = W->colptr[c]; p < W->colptr[c + 1]; ++p) s += W->A[p] * x[W->rowidx[p]];
    y[c] = s;
  }
}
/* ---- block-tridiagonal Cholesky of P + sigma I + A' diag(rho) A --------- */
static int bt_factor(Work* W, double sigma, const double* rho) {
  const int N = W->N;
  memset(W->Kd, 0, 8 * (size_t)N * 576);
  memset(W->Ko, 0, 8 * (size_t)N * 576);
  for (int c = 0; c < W->n; ++c) W->Kd[576 * W->stage[c] + 25 * W->loc[c]] += W->Pd[c] + sigma;
  for (int r = 0; r < W->m; ++r) {
    if (rho[r] == 0.0) continue;
    for (int a = W->rowptr[r]; a < W->rowptr[r + 1]; ++a)
      for (int b = W->rowptr[r]; b < W->rowptr[r + 1]; ++b) {
        int ca = W->colidx[a], cb = W->colidx[b];
        int sa = W->stage[ca], sb = W->stage[cb];
        double v = rho[r] * W->A[W->cscpos[a]] * W->A[W->cscpos[b]];
        if (sa == sb) W->Kd[576 * sa + 24 * W->loc[ca] + W->loc[cb]] += v;
        else if (sa == sb + 1) W->Ko[576 * sa + 24 * W->loc[ca] + W->loc[cb]] += v;
      }
  }
  /* in place: Kd[k] <- L_k (lower), Ko[k] <- L_{k,k-1} */
  for (int k = 0; k < N; ++k) {
    double* L = W->Kd + 576 * k;
    if (k > 0) {
      double* Lo = W->Ko + 576 * k;
      for (int i = 0; i < 24; ++i)
        for (int j = 0; j <= i; ++j) {
          double s = 0.0;
          for (int t = 0; t < 24; ++t) s += Lo[24 * i + t] * Lo[24 * j + t];
          L[24 * i + j] -= s;
        }
    }
    for (int j = 0; j < 24; ++j) {
      double d = L[25 * j];
      for (int t = 0; t < j; ++t) d -= L[24 * j + t] * L[24 * j + t];
      if (!(d > 0.0)) return -1;
      d = sqrt(d);
      L[25 * j] = d;
      for (int i = j + 1; i < 24; ++i) {
        double s = L[24 * i + j];
        for (int t = 0; t < j; ++t) s -= L[24 * i + t] * L[24 * j + t];
        L[24 * i + j] = s / d;
      }
    }
    for (int i = 0; i < 24; ++i)
      for (int j = i + 1; j < 24; ++j) L[24 * i + j] = 0.0;
    if (k + 1 < N) { /* L_{k+1,k} = K_{k+1,k} L_k^{-T}: row-wise forward solve */
      double* Lo = W->Ko + 576 * (k + 1);
      for (int i = 0; i < 24; ++i)
        for (int j = 0; j < 24; ++j) {
          double s = Lo[24 * i + j];
          for (int t = 0; t < j; ++t) s -= Lo[24 * i + t] * L[24 * j + t];
          Lo[24 * i + j] = s / L[25 * j];
        }
    }
  }
  return 0;
}

/* solve (P + sigma I + A'RA) out = b  (natural ordering) */
static void bt_solve(Work* W, const double* b, double* out) {
  const int N = W->N;
  double* t = W->tmpn; /* stage ordered */
  for (int c = 0; c < W->n; ++c) t[24 * W->stage[c] + W->loc[c]] = b[c];
  for (int k = 0; k < N; ++k) {
    double* v = t + 24 * k;
    const double* L = W->Kd + 576 * k;
    if (k > 0) {
      const double* Lo = W->Ko + 576 * k;
      const double* vp = t + 24 * (k - 1);
      for (int i = 0; i < 24; ++i) {
        double s = 0.0;
        for (int j = 0; j < 24; ++j) s += Lo[24 * i + j] * vp[j];
        v[i] -= s;
      }
    }
    for (int i = 0; i < 24; ++i) {
      double s = v[i];
      for (int j = 0; j < i; ++j) s -= L[24 * i + j] * v[j];
      v[i] = s / L[25 * i];
    }
  }
  for (int k = N - 1; k >= 0; --k) {
    double* v = t + 24 * k;
    const double* L = W->Kd + 576 * k;
    if (k + 1 < N) {
      const double* Lo = W->Ko + 576 * (k + 1);
      const double* vn = t + 24 * (k + 1);
      for (int j = 0; j < 24; ++j) {
        double s = 0.0;
        for (int i = 0; i < 24; ++i) s += Lo[24 * i + j] * vn[i];
        v[j] -= s;
      }
    }
    for (int i = 23; i >= 0; --i) {
      double s = v[i];
      for (int j = i + 1; j < 24; ++j) s -= L[24 * j + i] * v[j];
      v[i] = s / L[25 * i];
    }
  }
  for (int c = 0; c < W->n; ++c) out[c] = t[24 * W->stage[c] + W->loc[c]];
}

/* ---- OSQP pieces ---------------------------------------------------------- */
static void limit_scaling_vec(double* v, int n) {
  for (int i = 0; i < n; ++i) {
    if (v[i] < MIN_SCALING) v[i] = 1.0;
    else if (v[i] > MAX_SCALING) v[i] = MAX_SCALING;
  }
}
static double limit_scaling_scalar(double v) {
  if (v < MIN_SCALING) return 1.0;
  if (v > MAX_SCALING) return MAX_SCALING;
  return v;
}

static void scale_data(Work* W, int iters) {
  int n = W->n, m = W->m;
  W->c = 1.0;
  for (int i = 0; i < n; ++i) W->D[i] = 1.0;
  for (int i = 0; i < m; ++i) W->E[i] = 1.0;
  double* Dt = W->tmpn;
  double* Et = W->tmpm;
  for (int it = 0; it < iters; ++it) {
    for (int c = 0; c < n; ++c) {
      double v = fabs(W->Pd[c]);
      for (int p = W->colptr[c]; p < W->colptr[c + 1]; ++p) {
        double a = fabs(W->A[p]);
        if (a > v) v = a;
      }
      Dt[c] = v;
    }
    for (int r = 0; r < m; ++r) {
      double v = 0.0;
      for (int q = W->rowptr[r]; q < W->rowptr[r + 1]; ++q) {
        double a = fabs(W->A[W->cscpos[q]]);
        if (a > v) v = a;
      }
      Et[r] = v;
    }
    limit_scaling_vec(Dt, n);
    limit_scaling_vec(Et, m);
    for (int c = 0; c < n; ++c) Dt[c] = 1.0 / sqrt(Dt[c]);
    for (int r = 0; r < m; ++r) Et[r] = 1.0 / sqrt(Et[r]);
    for (int c = 0; c < n; ++c) {
      W->Pd[c] = Dt[c] * W->Pd[c] * Dt[c];
      for (int p = W->colptr[c]; p < W->colptr[c + 1]; ++p) W->A[p] = Et[W->rowidx[p]] * W->A[p] * Dt[c];
      W->D[c] *= Dt[c];
    }
    for (int r = 0; r < m; ++r) W->E[r] *= Et[r];
    /* cost scaling (q = 0 so its norm is limited to 1) */
    double mean = 0.0;
    for (int c = 0; c < n; ++c) mean += fabs(W->Pd[c]);
    mean /= n;
    double ct = mean > 1.0 ? mean : 1.0; /* max(mean, limit(|q|=0)=1) */
    ct = limit_scaling_scalar(ct);
    ct = 1.0 / ct;
    for (int c = 0; c < n; ++c) W->Pd[c] *= ct;
    W->c *= ct;
  }
}

static void set_rho_vec(Work* W, double rho) {
  for (int r = 0; r < W->m; ++r) {
    if (W->lo[r] < -OSQP_INFTY * MIN_SCALING && W->hi[r] > OSQP_INFTY * MIN_SCALING) {
      W->ctype[r] = -1; W->rho[r] = RHO_MIN;
    } else if (W->hi[r] - W->lo[r] < RHO_TOL) {
      W->ctype[r] = 1; W->rho[r] = RHO_EQ_OVER_RHO_INEQ * rho;
    } else {
      W->ctype[r] = 0; W->rho[r] = rho;
    }
  }
}

typedef struct { double pri_res, dua_res, eps_pri, eps_dua, s_pri, s_dua; } Info;

/* residuals at (x, z, y) (scaled vectors); also fills Ax, Px, Aty */
static void update_info(Work* W, const double* x, const double* z, const double* y,
                        const mpcq_params* p, Info* I) {
  int n = W->n, m = W->m;
  mat_vec(W, x, W->Ax);
  for (int c = 0; c < n; ++c) W->Px[c] = W->Pd[c] * x[c];
  mat_tvec(W, y, W->Aty);
  double* Einv = W->tmpm;
  double* Dinv = W->tmpn;
  for (int r = 0; r < m; ++r) Einv[r] = 1.0 / W->E[r];
  for (int c = 0; c < n; ++c) Dinv[c] = 1.0 / W->D[c];
  double pr = 0.0, nax = 0.0, nz = 0.0, spr = 0.0, snax = 0.0, snz = 0.0;
  for (int r = 0; r < m; ++r) {
    double d = W->Ax[r] - z[r];
    double a = fabs(Einv[r] * d); if (a > pr) pr = a;
    a = fabs(Einv[r] * W->Ax[r]); if (a > nax) nax = a;
    a = fabs(Einv[r] * z[r]); if (a > nz) nz = a;
    a = fabs(d); if (a > spr) spr = a;
    a = fabs(W->Ax[r]); if (a > snax) snax = a;
    a = fabs(z[r]); if (a > snz) snz = a;
  }
  double dr = 0.0, npx = 0.0, naty = 0.0, sdr = 0.0, snpx = 0.0, snaty = 0.0;
  for (int c = 0; c < n; ++c) {
    double d = W->Px[c] + 0.0 + W->Aty[c];
    double a = fabs(Dinv[c] * d); if (a > dr) dr = a;
    a = fabs(Dinv[c] * W->Px[c]); if (a > npx) npx = a;
    a = fabs(Dinv[c] * W->Aty[c]); if (a > naty) naty = a;
    a = fabs(d); if (a > sdr) sdr = a;
    a = fabs(W->Px[c]); if (a > snpx) snpx = a;
    a = fabs(W->Aty[c]); if (a > snaty) snaty = a;
  }
  double cinv = 1.0 / W->c;
  I->pri_res = pr;
  I->dua_res = cinv * dr;
  I->eps_pri = p->eps_abs + p->eps_rel * (nax > nz ? nax : nz);
  double md = npx > naty ? npx : naty; /* ||Dinv q|| = 0 */
  I->eps_dua = p->eps_abs + p->eps_rel * cinv * md;
  /* scaled, normalised residuals for the rho estimate */
  double pn = snax > snz ? snax : snz;
  double dn = snpx > snaty ? snpx : snaty;
  I->s_pri = spr / (pn + DIV_TOL);
  I->s_dua = sdr / (dn + DIV_TOL);
}

static int check_term(const Info* I, const mpcq_params* p, int approximate) {
  /* approximate check: eps_abs and eps_rel both x10, so the tolerance x10 */
  double f = approximate ? 10.0 : 1.0;
  (void)p;
  double eps_pri = f * I->eps_pri, eps_dua = f * I->eps_dua;
  return (I->pri_res < eps_pri) && (I->dua_res < eps_dua);
}

/* osqp 0.6 auxil.c is_primal_infeasible, on the scaled data and the last
 * iteration's delta_y: project delta_y onto the polar of the recession cone of
 * [l, u], then ||E dy|| > 0, u'max(dy, 0) + l'min(dy, 0) < eps ||E dy|| and
 * ||D^-1 A' dy|| < eps ||E dy||. */
static int is_primal_infeasible(Work* W, double eps) {
  const int m = W->m, n = W->n;
  double* dy = W->dy;
  for (int r = 0; r < m; ++r) {
    if (W->hi[r] > OSQP_INFTY * MIN_SCALING) {
      if (W->lo[r] < -OSQP_INFTY * MIN_SCALING) dy[r] = 0.0;
      else dy[r] = dy[r] < 0.0 ? dy[r] : 0.0;
    } else if (W->lo[r] < -OSQP_INFTY * MIN_SCALING) {
      dy[r] = dy[r] > 0.0 ? dy[r] : 0.0;
    }
  }
  double norm = 0.0;
  for (int r = 0; r < m; ++r) { double a = fabs(W->E[r] * dy[r]); if (a > norm) norm = a; }
  if (!(norm > DIV_TOL)) return 0;
  double ineq = 0.0;
  for (int r = 0; r < m; ++r)
    ineq += W->hi[r] * (dy[r] > 0.0 ? dy[r] : 0.0) + W->lo[r] * (dy[r] < 0.0 ? dy[r] : 0.0);
  if (!(ineq < eps * norm)) return 0;
  double* aty = W->tmpn2;
  mat_tvec(W, dy, aty);
  double na = 0.0;
  for (int c = 0; c < n; ++c) { double a = fabs(aty[c] / W->D[c]); if (a > na) na = a; }
  return na < eps * norm;
}

/* osqp 0.6 auxil.c is_dual_infeasible, on the last iteration's delta_x:
 * ||D dx|| > 0, q'dx < c eps ||D dx|| (q = 0), ||D^-1 P dx|| < c eps ||D dx|| and
 * every row with a finite bound keeps (E^-1 A dx) on its side within eps ||D dx||. */
static int is_dual_infeasible(Work* W, double eps) {
  const int m = W->m, n = W->n;
  const double* dx = W->dx;
  double norm = 0.0;
  for (int c = 0; c < n; ++c) { double a = fabs(W->D[c] * dx[c]); if (a > norm) norm = a; }
  if (!(norm > DIV_TOL)) return 0;
  if (!(0.0 < W->c * eps * norm)) return 0; /* q'dx = 0 */
  double np_ = 0.0;
  for (int c = 0; c < n; ++c) { double a = fabs(W->Pd[c] * dx[c] / W->D[c]); if (a > np_) np_ = a; }
  if (!(np_ < W->c * eps * norm)) return 0;
  double* adx = W->tmpm2;
  mat_vec(W, dx, adx);
  for (int r = 0; r < m; ++r) {
    const double v = adx[r] / W->E[r];
    if ((W->hi[r] < OSQP_INFTY * MIN_SCALING && v > eps * norm) ||
        (W->lo[r] > -OSQP_INFTY * MIN_SCALING && v < -eps * norm))
      return 0;
  }
  return 1;
}

/* osqp 0.6 check_termination: solved, else primal, else dual infeasible (each
 * infeasibility test only where its residual test failed); approximate = the
 * x10 tolerances of the max_iter exit.  Returns the status or 0. */
static int check_termination(Work* W, const Info* I, const mpcq_params* p, int approximate) {
  const double f = approximate ? 10.0 : 1.0;
  const int pri_ok = I->pri_res < f * I->eps_pri, dua_ok = I->dua_res < f * I->eps_dua;
  const int pinf = !pri_ok && is_primal_infeasible(W, f * p->eps_prim_inf);
  const int dinf = !dua_ok && is_dual_infeasible(W, f * p->eps_dual_inf);
  if (pri_ok && dua_ok) return approximate ? MPCQ_STATUS_SOLVED_INACCURATE : MPCQ_STATUS_SOLVED;
  if (pinf) return approximate ? MPCQ_STATUS_PRIMAL_INFEASIBLE_INACCURATE : MPCQ_STATUS_PRIMAL_INFEASIBLE;
  if (dinf) return approximate ? MPCQ_STATUS_DUAL_INFEASIBLE_INACCURATE : MPCQ_STATUS_DUAL_INFEASIBLE;
  return 0;
}

/* ---- polish (OSQP 0.6 polish.c restated in reduced form) ----------------
 * One round = OSQP's polish: guess the active set from (z, y) (lower-active if
 * z - l < -y, upper-active if u - z < y), solve the equality-constrained QP
 * [P + dI, Ar'; Ar, -dI] (reduced: (P + dI + Ar'Ar/d) x = -q + Ar'b/d), refine
 * against the unregularised KKT, project (z, y) onto the normal cone and keep
 * the result if it lowers the residuals.  polish_rounds > 1 repeats the guess
 * from the polished (Ax, y) (a primal-dual active-set iteration) until the set
 * repeats, keeping the round with the smallest max(pri_res, dua_res). */
static void polish_solve(Work* W, const mpcq_params* p, const int* act, const double* bred,
                         double* xp, double* yp, double* zp, double* r1, double* r2, double* rhs,
                         double* dx) {
  int n = W->n, m = W->m;
  double delta = p->delta;
  for (int r = 0; r < m; ++r) W->w[r] = act[r] ? bred[r] / delta : 0.0;
  mat_tvec(W, W->w, rhs);
  bt_solve(W, rhs, xp);
  mat_vec(W, xp, zp);
  for (int r = 0; r < m; ++r) yp[r] = act[r] ? (zp[r] - bred[r]) / delta : 0.0;
  for (int it = 0; it < p->polish_refine_iter; ++it) {
    for (int r = 0; r < m; ++r) W->w[r] = act[r] ? yp[r] : 0.0;
    mat_tvec(W, W->w, r1);
    for (int c = 0; c < n; ++c) r1[c] = -W->Pd[c] * xp[c] - r1[c];
    mat_vec(W, xp, zp);
    for (int r = 0; r < m; ++r) r2[r] = act[r] ? bred[r] - zp[r] : 0.0;
    for (int r = 0; r < m; ++r) W->w[r] = act[r] ? r2[r] / delta : 0.0;
    mat_tvec(W, W->w, rhs);
    for (int c = 0; c < n; ++c) rhs[c] += r1[c];
    bt_solve(W, rhs, dx);
    mat_vec(W, dx, zp);
    for (int c = 0; c < n; ++c) xp[c] += dx[c];
    for (int r = 0; r < m; ++r) if (act[r]) yp[r] += (zp[r] - r2[r]) / delta;
  }
  mat_vec(W, xp, zp);
}

static int polish(Work* W, const mpcq_params* p, Info* admm_info, double* x, double* z, double* y) {
  int n = W->n, m = W->m;
  double* rho = xalloc(8 * m);
  double* bred = xalloc(8 * m);
  int* act = xalloc(sizeof(int) * m);
  int* prev = xalloc(sizeof(int) * m);
  double *xp = xalloc(8 * n), *yp = xalloc(8 * m), *zp = xalloc(8 * m);
  double *zs = xalloc(8 * m), *ys = xalloc(8 * m);
  double *bx = xalloc(8 * n), *by = xalloc(8 * m), *bz = xalloc(8 * m);
  double *r1 = xalloc(8 * n), *r2 = xalloc(8 * m), *rhs = xalloc(8 * n), *dx = xalloc(8 * n);
  int ok = 0, have = 0;
  Info best;
  memset(&best, 0, sizeof(best));
  memcpy(zs, z, 8 * m);
  memcpy(ys, y, 8 * m);
  int rounds = p->polish_rounds > 0 ? p->polish_rounds : 1;
  for (int r = 0; r < m; ++r) prev[r] = 0;
  for (int rd = 0; rd < rounds; ++rd) {
    int same = 1;
    for (int r = 0; r < m; ++r) {
      int a = 0;
      if (rd == 0) { /* OSQP's guess (polish.c form_Ared) */
        if (zs[r] - W->lo[r] < -ys[r]) a = -1;
        else if (W->hi[r] - zs[r] < ys[r]) a = 1;
        /* equality rows stay in the set even when y is exactly 0 (the GPU
           factorisation divides by their rho) */
        if (a == 0 && W->hi[r] - W->lo[r] < RHO_TOL) a = 1;
      } else {       /* keep correctly signed active rows, add violated rows */
        const double tol = 1e-12;
        int eq = W->hi[r] - W->lo[r] < RHO_TOL;
        if (prev[r] == -1 && (ys[r] <= tol || eq)) a = -1;
        else if (prev[r] == 1 && (ys[r] >= -tol || eq)) a = 1;
        else if (zs[r] < W->lo[r] - tol) a = -1;
        else if (zs[r] > W->hi[r] + tol) a = 1;
      }
      if (a == -1) bred[r] = W->lo[r];
      if (a == 1) bred[r] = W->hi[r];
      if (rd > 0 && a != prev[r]) same = 0;
      act[r] = a;
      prev[r] = a;
      rho[r] = a ? 1.0 / p->delta : 0.0;
    }
    if (rd > 0 && same) break;
    if (bt_factor(W, p->delta, rho) != 0) break;
    polish_solve(W, p, act, bred, xp, yp, zp, r1, r2, rhs, dx);
    memcpy(zs, zp, 8 * m);
    memcpy(ys, yp, 8 * m);
    for (int r = 0; r < m; ++r) { /* project_normalcone */
      double t = zp[r] + yp[r];
      double zz = t < W->lo[r] ? W->lo[r] : (t > W->hi[r] ? W->hi[r] : t);
      zp[r] = zz;
      yp[r] = t - zz;
    }
    Info P;
    update_info(W, xp, zp, yp, p, &P);
    double sc = P.pri_res > P.dua_res ? P.pri_res : P.dua_res;
    double bs = best.pri_res > best.dua_res ? best.pri_res : best.dua_res;
    if (!have || sc < bs) {
      have = 1;
      best = P;
      memcpy(bx, xp, 8 * n); memcpy(bz, zp, 8 * m); memcpy(by, yp, 8 * m);
    }
  }
  if (have) {
    int good = (best.pri_res < admm_info->pri_res && best.dua_res < admm_info->dua_res) ||
               (best.pri_res < admm_info->pri_res && admm_info->dua_res < 1e-10) ||
               (best.dua_res < admm_info->dua_res && admm_info->pri_res < 1e-10);
    if (good) {
      memcpy(x, bx, 8 * n); memcpy(z, bz, 8 * m); memcpy(y, by, 8 * m);
      ok = 1;
    } else ok = -1;
  }
  free(rho); free(bred); free(act); free(prev); free(xp); free(yp); free(zp); free(zs); free(ys);
  free(bx); free(by); free(bz); free(r1); free(r2); free(rhs); free(dx);
  return ok;
}

/* info_out: [0] iterations, [1] rho updates (refactorisations beyond the
 * first), [2] polish status (0 not run, 1 ok, -1 rejected), [3] the ADMM's own
 * status before polish (polish = 2 may upgrade it to SOLVED) */
int oracle_qp_solve(const mpcq_params* p, int N, const double* Ax, const double* l,
                    const double* u, const double* warm_x, const double* warm_y,
                    const double* rho_in, double* x_out, double* y_out, int32_t* status,
                    int32_t* iters, double* rho_out, int32_t* info_out) {
  Work Wk;
  if (work_init(&Wk, N) != 0) { work_free(&Wk); return -1; }
  Work* W = &Wk;
  int n = W->n, m = W->m;
  int st = 0, it_done = 0, n_upd = 0, pol = 0, admm_st = 0;
  double rho = p->rho;
  /* data (MPC.py:236-288 cost; python osqp clamps bounds to +-OSQP_INFTY) */
  for (int c = 0; c < n; ++c) W->Pd[c] = (c < 12 * N) ? p->state_weights[c % 12] : p->force_weight;
  memcpy(W->A, Ax, 8 * (size_t)W->nnz);
  int finite = 1;
  for (int q = 0; q < W->nnz; ++q) if (!isfinite(Ax[q])) finite = 0;
  int ordered = 1;
  for (int r = 0; r < m; ++r) {
    double lo = l[r] < -OSQP_INFTY ? -OSQP_INFTY : l[r];
    double hi = u[r] > OSQP_INFTY ? OSQP_INFTY : u[r];
    if (isnan(lo) || isnan(hi)) finite = 0;
    if (lo > hi) ordered = 0; /* osqp validate_data / osqp_update_bounds reject l > u */
    W->lo[r] = lo; W->hi[r] = hi;
  }
  if (!finite) { st = MPCQ_STATUS_NONFINITE; goto out; }
  if (!ordered) { st = MPCQ_STATUS_BAD_BOUNDS; goto out; }
  if (p->scaling > 0) scale_data(W, p->scaling);
  else { for (int c = 0; c < n; ++c) W->D[c] = 1.0; for (int r = 0; r < m; ++r) W->E[r] = 1.0; W->c = 1.0; }
  for (int r = 0; r < m; ++r) { W->lo[r] *= W->E[r]; W->hi[r] *= W->E[r]; }
  rho = rho_in ? rho_in[0] : p->rho;
  rho = rho < RHO_MIN ? RHO_MIN : (rho > RHO_MAX ? RHO_MAX : rho);
  set_rho_vec(W, rho);
  if (warm_x) {
    for (int c = 0; c < n; ++c) W->x[c] = warm_x[c] / W->D[c];
    mat_vec(W, W->x, W->z);
  }
  if (warm_y)  /* dual_warm = 1: osqp's workspace y, kept as is; 0: osqp_warm_start_y scaling */
    for (int r = 0; r < m; ++r) W->y[r] = p->dual_warm ? warm_y[r] : W->c * warm_y[r] / W->E[r];
  if (bt_factor(W, p->sigma, W->rho) != 0) { st = MPCQ_STATUS_FACTOR_FAILED; goto out; }
  Info I;
  memset(&I, 0, sizeof(I));
  int can_check = 0;
  int iter;
  for (iter = 1; iter <= p->max_iter; ++iter) {
    memcpy(W->xp, W->x, 8 * n);
    memcpy(W->zp, W->z, 8 * m);
    for (int r = 0; r < m; ++r) W->w[r] = W->rho[r] * W->zp[r] - W->y[r];
    mat_tvec(W, W->w, W->rhs);
    for (int c = 0; c < n; ++c) W->rhs[c] += p->sigma * W->xp[c]; /* - q, q = 0 */
    bt_solve(W, W->rhs, W->xt);
    mat_vec(W, W->xt, W->zt);
    for (int c = 0; c < n; ++c) {
      W->x[c] = p->alpha * W->xt[c] + (1.0 - p->alpha) * W->xp[c];
      W->dx[c] = W->x[c] - W->xp[c]; /* osqp update_x: delta_x */
    }
    for (int r = 0; r < m; ++r) {
      double zr = p->alpha * W->zt[r] + (1.0 - p->alpha) * W->zp[r];
      double t = zr + (1.0 / W->rho[r]) * W->y[r]; /* osqp: rho_inv_vec .* y */
      double zz = t < W->lo[r] ? W->lo[r] : (t > W->hi[r] ? W->hi[r] : t);
      W->dy[r] = W->rho[r] * (zr - zz); /* osqp update_y: delta_y */
      W->y[r] = W->y[r] + W->dy[r];
      W->z[r] = zz;
    }
    can_check = p->check_termination > 0 && (iter % p->check_termination == 0);
    if (can_check) {
      update_info(W, W->x, W->z, W->y, p, &I);
      if (!(isfinite(I.pri_res) && isfinite(I.dua_res))) { st = MPCQ_STATUS_NONFINITE; break; }
      if ((st = check_termination(W, &I, p, 0)) != 0) break;
    }
    if (p->adaptive_rho && p->adaptive_rho_interval > 0 && iter % p->adaptive_rho_interval == 0) {
      if (!can_check) update_info(W, W->x, W->z, W->y, p, &I);
      double rn = rho * sqrt(I.s_pri / (I.s_dua + DIV_TOL));
      rn = rn < RHO_MIN ? RHO_MIN : (rn > RHO_MAX ? RHO_MAX : rn);
      if (rn > rho * p->adaptive_rho_tolerance || rn < rho / p->adaptive_rho_tolerance) {
        rho = rn;
        set_rho_vec(W, rho);
        if (bt_factor(W, p->sigma, W->rho) != 0) { st = MPCQ_STATUS_FACTOR_FAILED; break; }
        n_upd++;
      }
    }
  }
  it_done = iter > p->max_iter ? p->max_iter : iter;
  if (st == 0) {
    if (!can_check) {
      update_info(W, W->x, W->z, W->y, p, &I);
      st = check_termination(W, &I, p, 0);
    }
    if (st == 0) st = check_termination(W, &I, p, 1);
    if (st == 0) st = MPCQ_STATUS_MAX_ITER_REACHED;
  }
  admm_st = st;
  /* polish == 1: OSQP (only after SOLVED); polish == 2: also after an inaccurate
   * or max-iter exit, upgrading the status when the polished point meets eps. */
  if (p->polish && (st == MPCQ_STATUS_SOLVED ||
                    (p->polish >= 2 && (st == MPCQ_STATUS_SOLVED_INACCURATE ||
                                        st == MPCQ_STATUS_MAX_ITER_REACHED)))) {
    pol = polish(W, p, &I, W->x, W->z, W->y);
    if (pol == 1 && st != MPCQ_STATUS_SOLVED) {
      Info Q;
      update_info(W, W->x, W->z, W->y, p, &Q);
      if (check_term(&Q, p, 0)) st = MPCQ_STATUS_SOLVED;
    }
  }
out:
  if (admm_st == 0) admm_st = st; /* the data checks' exits */
  if (x_out) for (int c = 0; c < n; ++c) x_out[c] = W->D[c] * W->x[c];
  if (y_out) for (int r = 0; r < m; ++r) y_out[r] = p->dual_warm ? W->y[r] : W->E[r] * W->y[r] / W->c;
  if (st == MPCQ_STATUS_NONFINITE || st == MPCQ_STATUS_FACTOR_FAILED || st == MPCQ_STATUS_BAD_BOUNDS) {
    if (x_out) for (int c = 0; c < n; ++c) x_out[c] = NAN;
  }
  if (st == MPCQ_STATUS_PRIMAL_INFEASIBLE || st == MPCQ_STATUS_DUAL_INFEASIBLE ||
      st == MPCQ_STATUS_PRIMAL_INFEASIBLE_INACCURATE || st == MPCQ_STATUS_DUAL_INFEASIBLE_INACCURATE) {
    /* osqp store_solution: no solution, x = y = NaN (and a cold start next time) */
    if (x_out) for (int c = 0; c < n; ++c) x_out[c] = NAN;
    if (y_out) for (int r = 0; r < m; ++r) y_out[r] = NAN;
  }
  if (status) *status = st;
  if (iters) *iters = it_done;
  if (rho_out) *rho_out = rho;
  if (info_out) { info_out[0] = it_done; info_out[1] = n_upd; info_out[2] = pol; info_out[3] = admm_st; }
  work_free(W);
  return 0;
}

/* fused formulation + solve for a batch (OpenMP over instances); info [B][4]
 * (optional) as oracle_qp_solve's info_out. */
int oracle_solve_batch(const mpcq_params* p, int N, int64_t B, const double* xref,
                       const double* fsteps, int mode, double* f0, double* x_out,
                       int32_t* status, int32_t* iters, int32_t* info, int nthreads) {
  int32_t n, m, nnz;
  oracle_dims(N, &n, &m, &nnz);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel
  {
    double* Ax = malloc(8 * (size_t)nnz);
    double* l = malloc(8 * (size_t)m);
    double* u = malloc(8 * (size_t)m);
    double* x = malloc(8 * (size_t)n);
#pragma omp for schedule(dynamic, 1)
    for (int64_t b = 0; b < B; ++b) {
      int32_t st = 0, it = 0, inf4[4] = {0, 0, 0, 0};
      int fs = oracle_formulate(p, N, xref + b * 12 * (N + 1), fsteps + b * 260, mode, Ax, l, u);
      if (fs != 0) {
        st = fs;
        inf4[3] = fs;
        for (int c = 0; c < n; ++c) x[c] = NAN;
      } else {
        oracle_qp_solve(p, N, Ax, l, u, NULL, NULL, NULL, x, NULL, &st, &it, NULL, inf4);
      }
      if (info) memcpy(info + 4 * b, inf4, sizeof inf4);
      if (f0) memcpy(f0 + 12 * b, x + 12 * N, 12 * 8);
      if (x_out) memcpy(x_out + b * n, x, 8 * (size_t)n);
      if (status) status[b] = st;
      if (iters) iters[b] = it;
    }
    free(Ax); free(l); free(u); free(x);
  }
  return 0;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
