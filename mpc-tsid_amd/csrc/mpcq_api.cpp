// mpcq_api.cpp — host side of the C ABI declared in include/mpcq.h.
//
// Owns HIP contexts, device staging buffers for host-pointer calls, stream
// and event handling.  All numerics run in the HIP kernels
// (mpcq_kernels.hip); there is no CPU fallback: a missing device is an error.
#include <math.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>

#include "mpcq_internal.h"

struct mpcq_ctx {
  int device = 0;
  int N = 0;
  mpcq_params p{};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  void* arena = nullptr;
  size_t arena_bytes = 0;
  void* work = nullptr;  // engine workspace (horizons beyond 32 stages)
  size_t work_bytes = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool have_form = false, have_solve = false;
  uint64_t* stamps = nullptr;
  // MPCQ_FLAG_ORDER_BY_CLASS: the class table (sum of iterations, count per slot) and the
  // per-instance scratch (class slot, dispatch order, iteration counts when the caller
  // passes none)
  uint64_t* cls_sum = nullptr;
  uint32_t* cls_cnt = nullptr;
  int32_t* ord_buf = nullptr;
  int64_t ord_cap = 0;
  // sliced solves (mpcq_set_slice): the slice length (0: off), the suspended instances'
  // iterates (mpcq::res_lanes(N) x 8 doubles, rho, key, 4 counters each), the resumed launch's
  // dispatch list (B int32, of 3 B: two once held alternating lists) and a status scratch, the
  // resumed launch's workgroup count (device)
  int32_t slice_iters = 0;
  double* res = nullptr;
  double* res_rho = nullptr;
  double* res_key = nullptr;
  int32_t* res_i = nullptr;
  int32_t* sl_buf = nullptr;
  int64_t sl_cap = 0;
  int32_t* sl_count = nullptr;
};

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(MPCQ_E_DEVICE, "%s failed: %s", #expr, hipGetErrorString(e_));        \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int check_params(const mpcq_params* p) {
  if (!p) return fail(MPCQ_E_INVALID, "params is NULL");
  if (!(p->dt > 0) || !(p->mass > 0)) return fail(MPCQ_E_INVALID, "dt and mass must be > 0");
  if (!(p->rho > 0) || !(p->sigma > 0) || !(p->alpha > 0 && p->alpha < 2))
    return fail(MPCQ_E_INVALID, "need rho > 0, sigma > 0, 0 < alpha < 2");
  if (!(p->eps_abs >= 0) || !(p->eps_rel >= 0)) return fail(MPCQ_E_INVALID, "eps must be >= 0");
  if (!(p->eps_prim_inf >= 0) || !(p->eps_dual_inf >= 0))
    return fail(MPCQ_E_INVALID, "eps_prim_inf / eps_dual_inf must be >= 0");
  if (p->dual_warm != 0 && p->dual_warm != 1) return fail(MPCQ_E_INVALID, "dual_warm must be 0 or 1");
  if (p->max_iter < 1 || p->check_termination < 0 || p->scaling < 0 || p->adaptive_rho_interval < 0)
    return fail(MPCQ_E_INVALID, "max_iter >= 1, check_termination/scaling/interval >= 0");
  if (!(p->adaptive_rho_tolerance >= 1)) return fail(MPCQ_E_INVALID, "adaptive_rho_tolerance >= 1");
  if (!(p->force_weight > 0)) return fail(MPCQ_E_INVALID, "force_weight must be > 0");
  for (int i = 0; i < 12; ++i)
    if (!(p->state_weights[i] > 0)) return fail(MPCQ_E_INVALID, "state weights must be > 0");
  if (p->polish < 0 || p->polish > 2) return fail(MPCQ_E_INVALID, "polish must be 0, 1 or 2");
  if (p->polish && (!(p->delta > 0) || p->polish_refine_iter < 0 || p->polish_rounds < 1))
    return fail(MPCQ_E_INVALID, "polish needs delta > 0, polish_refine_iter >= 0, polish_rounds >= 1");
  return MPCQ_OK;
}

// Stage the listed host arrays into the context arena.  Each entry: host
// pointer, byte count, direction (1 = in, 2 = out).  Returns device pointers.
struct Xfer {
  const void* host_in;
  void* host_out;
  size_t bytes;
  void* dev;
};

int ensure_arena(mpcq_ctx* c, size_t bytes) {
  if (bytes <= c->arena_bytes) return MPCQ_OK;
  if (c->arena) HIP_TRY(hipFree(c->arena));
  c->arena = nullptr;
  c->arena_bytes = 0;
  size_t want = bytes + bytes / 4;
  if (hipMalloc(&c->arena, want) != hipSuccess) {
    c->arena = nullptr;
    return fail(MPCQ_E_NOMEM, "hipMalloc(%zu) failed", want);
  }
  c->arena_bytes = want;
  return MPCQ_OK;
}

// The engine's per-instance workspace (mpcq::work_doubles(N), zero up to 32 stages).
int ensure_work(mpcq_ctx* c, int64_t B, double** out) {
  *out = nullptr;
  const size_t bytes = (size_t)mpcq::work_doubles(c->N) * 8 * (size_t)B;
  if (bytes == 0) return MPCQ_OK;
  if (bytes > c->work_bytes) {
    if (c->work) {
      HIP_TRY(hipStreamSynchronize(c->stream));  // a queued launch may still use it
      HIP_TRY(hipFree(c->work));
    }
    c->work = nullptr;
    c->work_bytes = 0;
    if (hipMalloc(&c->work, bytes) != hipSuccess) {
      c->work = nullptr;
      return fail(MPCQ_E_NOMEM, "hipMalloc(%zu) for the engine workspace failed", bytes);
    }
    // zeroed once, as a guard only: no kernel reads a workspace slot it has not
    // written earlier in the same launch (DESIGN.md §4.1 "LDS hygiene"; the suite
    // passes on a build without the LDS zeroing either)
    HIP_TRY(hipMemsetAsync(c->work, 0, bytes, c->stream));
    c->work_bytes = bytes;
  }
  *out = (double*)c->work;
  return MPCQ_OK;
}

// MPCQ_FLAG_ORDER_BY_CLASS scratch: the class table (zeroed once, kept for the context's
// life) and 3 B int32 (class slots, order, iteration counts)
int ensure_order(mpcq_ctx* c, int64_t B) {
  const int slots = mpcq::class_table_slots();
  if (!c->cls_sum) {
    void* tab = nullptr;
    const size_t tb = (size_t)slots * (8 + 4);
    if (hipMalloc(&tab, tb) != hipSuccess) return fail(MPCQ_E_NOMEM, "hipMalloc(%zu) for the class table failed", tb);
    c->cls_sum = (uint64_t*)tab;
    c->cls_cnt = (uint32_t*)((char*)tab + (size_t)slots * 8);
    HIP_TRY(hipMemsetAsync(tab, 0, tb, c->stream));
  }
  if (B > c->ord_cap) {
    if (c->ord_buf) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(hipFree(c->ord_buf));
    }
    c->ord_buf = nullptr;
    c->ord_cap = 0;
    if (hipMalloc(&c->ord_buf, (size_t)B * 12) != hipSuccess) {
      c->ord_buf = nullptr;
      return fail(MPCQ_E_NOMEM, "hipMalloc(%zu) for the dispatch order failed", (size_t)B * 12);
    }
    c->ord_cap = B;
  }
  return MPCQ_OK;
}

int stage(mpcq_ctx* c, Xfer* xs, int nx) {
  size_t tot = 0;
  for (int i = 0; i < nx; ++i)
    if (xs[i].host_in || xs[i].host_out) tot += (xs[i].bytes + 255) & ~size_t(255);
  int rc = ensure_arena(c, tot);
  if (rc) return rc;
  size_t off = 0;
  for (int i = 0; i < nx; ++i) {
    xs[i].dev = nullptr;
    if (!(xs[i].host_in || xs[i].host_out)) continue;
    xs[i].dev = (char*)c->arena + off;
    off += (xs[i].bytes + 255) & ~size_t(255);
    if (xs[i].host_in)
      HIP_TRY(hipMemcpyAsync(xs[i].dev, xs[i].host_in, xs[i].bytes, hipMemcpyHostToDevice, c->stream));
  }
  return MPCQ_OK;
}

int unstage(mpcq_ctx* c, Xfer* xs, int nx) {
  for (int i = 0; i < nx; ++i)
    if (xs[i].host_out)
      HIP_TRY(hipMemcpyAsync(xs[i].host_out, xs[i].dev, xs[i].bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPCQ_OK;
}

int check_ctx(mpcq_ctx* c, int64_t batch) {
  if (!c) return fail(MPCQ_E_INVALID, "ctx is NULL");
  if (batch < 0 || batch > (int64_t)0x7fffffff) return fail(MPCQ_E_INVALID, "bad batch %lld", (long long)batch);
  return MPCQ_OK;
}

// Sliced-solve scratch (mpcq_set_slice): the suspended iterates, the dispatch lists, the count
int ensure_slice(mpcq_ctx* c, int64_t B) {
  if (!c->sl_count) {
    if (hipMalloc(&c->sl_count, 4) != hipSuccess) {
      c->sl_count = nullptr;
      return fail(MPCQ_E_NOMEM, "hipMalloc(4) for the slice count failed");
    }
  }
  if (B > c->sl_cap) {
    if (c->res) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(hipFree(c->res));
      HIP_TRY(hipFree(c->sl_buf));
    }
    c->res = nullptr;
    c->sl_buf = nullptr;
    c->sl_cap = 0;
    const size_t rb = (size_t)B * (8 * (size_t)mpcq::res_lanes(c->N) + 3) * 8 + (size_t)B * 32;
    if (hipMalloc(&c->res, rb) != hipSuccess) {
      c->res = nullptr;
      return fail(MPCQ_E_NOMEM, "hipMalloc(%zu) for the suspended iterates failed", rb);
    }
    if (hipMalloc(&c->sl_buf, (size_t)B * 12) != hipSuccess) {
      c->sl_buf = nullptr;
      return fail(MPCQ_E_NOMEM, "hipMalloc(%zu) for the slice lists failed", (size_t)B * 12);
    }
    c->res_rho = c->res + (size_t)B * 8 * (size_t)mpcq::res_lanes(c->N);
    c->res_key = c->res_rho + B;
    c->res_i = (int32_t*)(c->res_key + 2 * B);
    c->sl_cap = B;
  }
  return MPCQ_OK;
}

}  // namespace

extern "C" {

int mpcq_abi_version(void) { return MPCQ_ABI_VERSION; }

// Reference constants: MPC.py:25-39 (dt from main.py:20, mass, gI, mu), 67-70
// (footholds), 201 (g), 228 (fz_max), 255-275 (weights); OSQP settings
// MPC.py:414-416 + osqp 0.6 defaults.
void mpcq_default_params(mpcq_params* p) {
  if (!p) return;
  memset(p, 0, sizeof(*p));
  p->dt = 0.02;
  p->mass = 2.50000279;
  const double gI[9] = {3.09249e-2, -8.00101e-7, 1.865287e-5, -8.00101e-7, 5.106100e-2,
                        1.245813e-4, 1.865287e-5, 1.245813e-4, 6.939757e-2};
  memcpy(p->gI, gI, sizeof(gI));
  p->mu = 0.9;
  p->fz_max = 25.0;
  p->gravity = 9.81;
  const double w[12] = {0.1, 0.1, 1.0, 0.11, 0.11, 0.11, 2.0 * sqrt(0.1), 2.0 * sqrt(0.1),
                        2.0 * sqrt(1.0), 0.05 * sqrt(0.11), 0.05 * sqrt(0.11), 0.05 * sqrt(0.11)};
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

int mpcq_dims(int N, int32_t* n, int32_t* m, int32_t* nnz) {
  if (N < 2) return fail(MPCQ_E_INVALID, "n_steps must be >= 2");
  if (n) *n = 24 * N;
  if (m) *m = 44 * N;
  if (nnz) *nnz = 126 * N - 18;
  return MPCQ_OK;
}

// CSC pattern of the dense matrix built by MPC.create_ML (MPC.py:103-151):
// state columns (-I of dynamics row k, A of dynamics row k+1), then per stage,
// foot and component the force column (dt/m row, B rows 9-11, swing row,
// friction rows).
int mpcq_pattern(int N, int32_t* indptr, int32_t* indices) {
  if (N < 2 || !indptr || !indices) return fail(MPCQ_E_INVALID, "bad arguments");
  int pos = 0;
  for (int c = 0; c < 12 * N; ++c) {
    const int k = c / 12, i = c % 12;
    indptr[c] = pos;
    indices[pos++] = c;
    if (k < N - 1) {
      if (i >= 6) indices[pos++] = 12 * (k + 1) + i - 6;
      indices[pos++] = 12 * (k + 1) + i;
    }
  }
  for (int k = 0; k < N; ++k)
    for (int f = 0; f < 4; ++f)
      for (int c = 0; c < 3; ++c) {
        indptr[12 * N + 12 * k + 3 * f + c] = pos;
        indices[pos++] = 12 * k + 6 + c;
        for (int r = 9; r < 12; ++r) indices[pos++] = 12 * k + r;
        indices[pos++] = 12 * N + 12 * k + 3 * f + c;
        const int fr = 24 * N + 20 * k + 5 * f;
        if (c == 0) { indices[pos++] = fr; indices[pos++] = fr + 1; }
        else if (c == 1) { indices[pos++] = fr + 2; indices[pos++] = fr + 3; }
        else for (int t = 0; t < 5; ++t) indices[pos++] = fr + t;
      }
  indptr[24 * N] = pos;
  return MPCQ_OK;
}

int mpcq_supported_horizons(int32_t* out, int cap) { return mpcq::supported_horizons(out, cap); }

const char* mpcq_last_error(void) { return g_err.c_str(); }

int mpcq_create(int device, int n_steps, const mpcq_params* params, mpcq_ctx** out) {
  if (!out) return fail(MPCQ_E_INVALID, "out is NULL");
  *out = nullptr;
  if (!mpcq::horizon_supported(n_steps))
    return fail(MPCQ_E_UNSUPPORTED, "horizon N=%d not compiled in (supported: 4 <= N <= 64)", n_steps);
  mpcq_params p;
  if (params) p = *params;
  else mpcq_default_params(&p);
  int rc = check_params(&p);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(MPCQ_E_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(MPCQ_E_INVALID, "device %d out of range (%d)", device, ndev);
  DeviceGuard g(device);
  mpcq_ctx* c = new mpcq_ctx();
  c->device = device;
  c->N = n_steps;
  c->p = p;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(MPCQ_E_DEVICE, "hipStreamCreate failed");
  }
  c->stream = c->own_stream;
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) {
      mpcq_destroy(c);
      return fail(MPCQ_E_DEVICE, "hipEventCreate failed");
    }
  *out = c;
  return MPCQ_OK;
}

int mpcq_destroy(mpcq_ctx* c) {
  if (!c) return MPCQ_OK;
  DeviceGuard g(c->device);
  if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
  if (c->arena) (void)hipFree(c->arena);
  if (c->work) (void)hipFree(c->work);
  if (c->cls_sum) (void)hipFree(c->cls_sum);
  if (c->ord_buf) (void)hipFree(c->ord_buf);
  if (c->res) (void)hipFree(c->res);
  if (c->sl_buf) (void)hipFree(c->sl_buf);
  if (c->sl_count) (void)hipFree(c->sl_count);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return MPCQ_OK;
}

int mpcq_set_stream(mpcq_ctx* c, void* stream) {
  if (!c) return fail(MPCQ_E_INVALID, "ctx is NULL");
  c->stream = stream ? (hipStream_t)stream : c->own_stream;
  return MPCQ_OK;
}

int mpcq_set_slice(mpcq_ctx* c, int32_t slice_iters) {
  if (!c) return fail(MPCQ_E_INVALID, "ctx is NULL");
  if (slice_iters < 0) return fail(MPCQ_E_INVALID, "slice_iters must be >= 0");
  c->slice_iters = slice_iters;
  return MPCQ_OK;
}

int mpcq_last_kernel_ms(mpcq_ctx* c, double* fms, double* sms) {
  if (!c) return fail(MPCQ_E_INVALID, "ctx is NULL");
  DeviceGuard g(c->device);
  float ms = 0.f;
  if (fms) {
    *fms = -1.0;
    if (c->have_form) {
      HIP_TRY(hipEventSynchronize(c->ev[1]));
      HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
      *fms = ms;
    }
  }
  if (sms) {
    *sms = -1.0;
    if (c->have_solve) {
      HIP_TRY(hipEventSynchronize(c->ev[3]));
      HIP_TRY(hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
      *sms = ms;
    }
  }
  return MPCQ_OK;
}

int mpcq_formulate_batch(mpcq_ctx* c, int64_t B, const double* xref, const double* fsteps, int mode,
                         double* Ax, double* l, double* u, int32_t* status, uint32_t flags) {
  int rc = check_ctx(c, B);
  if (rc) return rc;
  if (!xref || !fsteps || !Ax || !l || !u) return fail(MPCQ_E_INVALID, "NULL array");
  if (mode != MPCQ_MODE_UPDATE && mode != MPCQ_MODE_SETUP) return fail(MPCQ_E_INVALID, "bad mode");
  if (B == 0) return MPCQ_OK;
  DeviceGuard g(c->device);
  const int N = c->N;
  const size_t n12 = 12 * (N + 1), nnz = 126 * N - 18, m = 44 * N;
  mpcq::LaunchArgs a{};
  a.batch = B;
  a.mode = mode;
  const bool dev = flags & MPCQ_FLAG_DEVICE_PTRS;
  Xfer xs[6] = {{xref, nullptr, B * n12 * 8, nullptr}, {fsteps, nullptr, (size_t)B * 260 * 8, nullptr},
                {nullptr, Ax, B * nnz * 8, nullptr},   {nullptr, l, B * m * 8, nullptr},
                {nullptr, u, B * m * 8, nullptr},      {nullptr, status, (size_t)B * 4, nullptr}};
  if (!dev) {
    rc = stage(c, xs, 6);
    if (rc) return rc;
    a.xref = (const double*)xs[0].dev; a.fsteps = (const double*)xs[1].dev;
    a.Ax_out = (double*)xs[2].dev; a.l_out = (double*)xs[3].dev; a.u_out = (double*)xs[4].dev;
    a.status = (int32_t*)xs[5].dev;
  } else {
    a.xref = xref; a.fsteps = fsteps; a.Ax_out = Ax; a.l_out = l; a.u_out = u; a.status = status;
  }
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  HIP_TRY(mpcq::launch_formulate(N, c->p, a, c->stream));
  HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  c->have_form = true;
  if (!dev) return unstage(c, xs, 6);
  if (!(flags & MPCQ_FLAG_ASYNC)) HIP_TRY(hipStreamSynchronize(c->stream));
  return MPCQ_OK;
}

static int solve_common(mpcq_ctx* c, int64_t B, bool fused, const double* xref, const double* fsteps,
                        int mode, const double* Ax, const double* l, const double* u,
                        const double* warm_x, const double* warm_y, const double* rho_in, double* f0,
                        double* x, double* y, int32_t* status, int32_t* iters, double* rho_out,
                        int32_t* info, uint32_t flags) {
  int rc = check_ctx(c, B);
  if (rc) return rc;
  if (B == 0) return MPCQ_OK;
  DeviceGuard g(c->device);
  const int N = c->N;
  const size_t n = 24 * N, m = 44 * N, nnz = 126 * N - 18, n12 = 12 * (N + 1);
  mpcq::LaunchArgs a{};
  a.batch = B;
  a.mode = mode;
  const bool dev = flags & MPCQ_FLAG_DEVICE_PTRS;
  enum { XR, FS, AX, L, U, WX, WY, RI, F0, X, Y, ST, IT, RO, IN, NX };
  Xfer xs[NX] = {
      {xref, nullptr, B * n12 * 8, nullptr},      {fsteps, nullptr, (size_t)B * 260 * 8, nullptr},
      {Ax, nullptr, B * nnz * 8, nullptr},        {l, nullptr, B * m * 8, nullptr},
      {u, nullptr, B * m * 8, nullptr},           {warm_x, nullptr, B * n * 8, nullptr},
      {warm_y, nullptr, B * m * 8, nullptr},      {rho_in, nullptr, (size_t)B * 8, nullptr},
      {nullptr, f0, (size_t)B * 12 * 8, nullptr}, {nullptr, x, B * n * 8, nullptr},
      {nullptr, y, B * m * 8, nullptr},           {nullptr, status, (size_t)B * 4, nullptr},
      {nullptr, iters, (size_t)B * 4, nullptr},   {nullptr, rho_out, (size_t)B * 8, nullptr},
      {nullptr, info, (size_t)B * 16, nullptr}};
  if (!dev) {
    rc = stage(c, xs, NX);
    if (rc) return rc;
    a.xref = (const double*)xs[XR].dev; a.fsteps = (const double*)xs[FS].dev;
    a.Ax = (const double*)xs[AX].dev; a.l = (const double*)xs[L].dev; a.u = (const double*)xs[U].dev;
    a.warm_x = (const double*)xs[WX].dev; a.warm_y = (const double*)xs[WY].dev;
    a.rho_in = (const double*)xs[RI].dev;
    a.f0 = (double*)xs[F0].dev; a.x = (double*)xs[X].dev; a.y = (double*)xs[Y].dev;
    a.status = (int32_t*)xs[ST].dev; a.iters = (int32_t*)xs[IT].dev; a.rho_out = (double*)xs[RO].dev;
    a.info = (int32_t*)xs[IN].dev;
  } else {
    a.xref = xref; a.fsteps = fsteps; a.Ax = Ax; a.l = l; a.u = u;
    a.warm_x = warm_x; a.warm_y = warm_y; a.rho_in = rho_in;
    a.f0 = f0; a.x = x; a.y = y; a.status = status; a.iters = iters; a.rho_out = rho_out;
    a.info = info;
  }
  a.stamps = c->stamps;
  rc = ensure_work(c, B, &a.work);
  if (rc) return rc;
  const bool by_class = fused && (flags & MPCQ_FLAG_ORDER_BY_CLASS);
  int32_t *cls = nullptr, *its = a.iters;
  if (by_class) {
    if (B > INT32_MAX) return fail(MPCQ_E_INVALID, "MPCQ_FLAG_ORDER_BY_CLASS: batch > INT32_MAX");
    rc = ensure_order(c, B);
    if (rc) return rc;
    cls = c->ord_buf;
    int32_t* order = c->ord_buf + B;
    if (!its) its = a.iters = c->ord_buf + 2 * B;  // (the engine writes them; the caller asked for none)
    HIP_TRY(mpcq::launch_class_order(a.fsteps, B, cls, c->cls_sum, c->cls_cnt, order, c->stream));
    a.order = order;
  }
  // sliced (mpcq_set_slice, beyond 16 stages): the first launch suspends every instance still
  // running after slice_iters iterations; a second launch resumes the suspended ones, the
  // farthest from convergence (the iterations left, extrapolated from the residuals' decay)
  // first, and runs them to their end.  (Re-slicing the second launch too was slower: C3 39.0 k
  // against 44.1 k QP/s at 1200, profiles/r06r_*.)
  const bool sliced = c->slice_iters > 0 && c->slice_iters < c->p.max_iter && (N > 16 || getenv("MPCQ_SLICE16"));
  if (sliced) {
    rc = ensure_slice(c, B);
    if (rc) return rc;
    a.slice_iters = c->slice_iters;
    a.res = c->res;
    a.res_rho = c->res_rho;
    a.res_key = c->res_key;
    a.res_i = c->res_i;
    if (!a.status) a.status = c->sl_buf + 2 * B;  // (the slices' statuses; the caller asked for none)
  }
  HIP_TRY(hipEventRecord(c->ev[2], c->stream));
  HIP_TRY(mpcq::launch_solve(N, fused, c->p, a, c->stream));
  if (sliced) {  // the suspended instances, farthest from convergence first, resumed once to their end
    // (the resumed launch is sized for the whole batch and reads the count from the device:
    // workgroups past it return at once -- no host round trip, the call stays asynchronous)
    int32_t* list = c->sl_buf;
    HIP_TRY(mpcq::launch_suspended(a.order, B, a.status, c->res_key, list, c->sl_count, c->stream));
    mpcq::LaunchArgs r = a;
    r.order = list;
    r.batch_dev = c->sl_count;
    r.resume = 1;
    r.slice_iters = 0;
    HIP_TRY(mpcq::launch_solve(N, fused, c->p, r, c->stream));
  }
  HIP_TRY(hipEventRecord(c->ev[3], c->stream));
  if (by_class) HIP_TRY(mpcq::launch_class_learn(cls, its, B, c->cls_sum, c->cls_cnt, c->stream));
  c->have_solve = true;
  if (!dev) return unstage(c, xs, NX);
  if (!(flags & MPCQ_FLAG_ASYNC)) HIP_TRY(hipStreamSynchronize(c->stream));
  return MPCQ_OK;
}

int mpcq_qp_solve_batch(mpcq_ctx* c, int64_t B, const double* Ax, const double* l, const double* u,
                        const double* warm_x, const double* warm_y, const double* rho_in, double* x,
                        double* y, int32_t* status, int32_t* iters, double* rho_out, int32_t* info,
                        uint32_t flags) {
  if (!Ax || !l || !u) return fail(MPCQ_E_INVALID, "Ax, l, u are required");
  return solve_common(c, B, false, nullptr, nullptr, 0, Ax, l, u, warm_x, warm_y, rho_in, nullptr, x,
                      y, status, iters, rho_out, info, flags);
}

int mpcq_solve_batch(mpcq_ctx* c, int64_t B, const double* xref, const double* fsteps, int mode,
                     const double* warm_x, const double* warm_y, const double* rho_in, double* f0,
                     double* x, double* y, double* rho_out, int32_t* status, int32_t* iters,
                     int32_t* info, uint32_t flags) {
  if (!xref || !fsteps) return fail(MPCQ_E_INVALID, "xref, fsteps are required");
  if (mode != MPCQ_MODE_UPDATE && mode != MPCQ_MODE_SETUP) return fail(MPCQ_E_INVALID, "bad mode");
  return solve_common(c, B, true, xref, fsteps, mode, nullptr, nullptr, nullptr, warm_x, warm_y,
                      rho_in, f0, x, y, status, iters, rho_out, info, flags);
}

// FootstepPlanner constants (FootstepPlanner.py:18-52, 316-322, 376; processing.py:131).
void mpcq_default_planner_params(mpcq_planner_params* pp) {
  if (!pp) return;
  memset(pp, 0, sizeof(*pp));
  pp->dt = 0.02;
  pp->T_gait = 0.32;
  pp->h_ref = 0.2027682;
  pp->k_feedback = 0.03;
  pp->L = 0.12;
  pp->g = 9.81;
  pp->t_stance = 0.16;
  pp->cmd_threshold = 0.05;
  const double sh[8] = {0.19, 0.19, -0.19, -0.19, 0.15005, -0.15005, 0.15005, -0.15005};
  memcpy(pp->shoulders, sh, sizeof(sh));
  const double ro[8] = {0.14, 0.14, -0.14, -0.14, 0.12, -0.12, 0.12, -0.12};
  memcpy(pp->reduced_offset, ro, sizeof(ro));
}

int mpcq_plan_batch(mpcq_ctx* c, const mpcq_planner_params* pp, int64_t B, uint32_t ops, int k,
                    const double* state, const double* v_cur, const double* h, const double* l_feet,
                    const double* v_ref, const int32_t* reduced, double* gait, int32_t* rot_flag,
                    double* h_rot, double* xref, double* fsteps, int32_t* status, uint32_t flags) {
  int rc = check_ctx(c, B);
  if (rc) return rc;
  if (ops == 0 || (ops & ~(uint32_t)MPCQ_PLAN_TICK)) return fail(MPCQ_E_INVALID, "ops must be MPCQ_PLAN_* bits");
  if (!gait || !v_ref || !state) return fail(MPCQ_E_INVALID, "gait, state and v_ref are required");
  if ((ops & MPCQ_PLAN_FOOTSTEPS) && (!l_feet || !fsteps))
    return fail(MPCQ_E_INVALID, "MPCQ_PLAN_FOOTSTEPS needs l_feet and fsteps");
  if ((ops & MPCQ_PLAN_REFSTATES) && (!rot_flag || !h_rot || !xref))
    return fail(MPCQ_E_INVALID, "MPCQ_PLAN_REFSTATES needs rot_flag, h_rot and xref");
  mpcq_planner_params P;
  if (pp) P = *pp;
  else mpcq_default_planner_params(&P);
  if (!(P.dt > 0) || !(P.g > 0) || !(P.T_gait > P.dt)) return fail(MPCQ_E_INVALID, "planner needs dt > 0, g > 0, T_gait > dt");
  if (B == 0) return MPCQ_OK;
  DeviceGuard g(c->device);
  const int N = c->N;
  const size_t n12 = 12 * (N + 1);
  mpcq::PlanArgs a{};
  a.batch = B;
  a.N = N;
  a.ops = ops;
  a.k = k;
  const bool dev = flags & MPCQ_FLAG_DEVICE_PTRS;
  const bool fo = ops & MPCQ_PLAN_FOOTSTEPS, rs = ops & MPCQ_PLAN_REFSTATES;
  enum { ST, VC, H, LF, VR, RD, GA, RF, HR, XR, FS, SS, NX };
  // in/out buffers are staged both ways (host_in and host_out both set)
  Xfer xs[NX] = {{state, nullptr, (size_t)B * 96, nullptr},
                 {v_cur, nullptr, (size_t)B * 48, nullptr},
                 {h, nullptr, (size_t)B * 8, nullptr},
                 {fo ? l_feet : nullptr, nullptr, (size_t)B * 96, nullptr},
                 {v_ref, nullptr, (size_t)B * 48, nullptr},
                 {reduced, nullptr, (size_t)B * 4, nullptr},
                 {gait, gait, (size_t)B * 800, nullptr},
                 {rs ? rot_flag : nullptr, rs ? rot_flag : nullptr, (size_t)B * 4, nullptr},
                 {rs ? h_rot : nullptr, rs ? h_rot : nullptr, (size_t)B * 8, nullptr},
                 {rs ? xref : nullptr, rs ? xref : nullptr, B * n12 * 8, nullptr},
                 // fsteps: staged in as well so a BAD_GAIT instance keeps the caller's values
                 {fo ? fsteps : nullptr, fo ? fsteps : nullptr, (size_t)B * 260 * 8, nullptr},
                 {nullptr, status, (size_t)B * 4, nullptr}};
  if (!dev) {
    rc = stage(c, xs, NX);
    if (rc) return rc;
    a.state = (const double*)xs[ST].dev; a.v_cur = (const double*)xs[VC].dev; a.h = (const double*)xs[H].dev;
    a.l_feet = (const double*)xs[LF].dev; a.v_ref = (const double*)xs[VR].dev;
    a.reduced = (const int32_t*)xs[RD].dev; a.gait = (double*)xs[GA].dev; a.rot_flag = (int32_t*)xs[RF].dev;
    a.h_rot = (double*)xs[HR].dev; a.xref = (double*)xs[XR].dev; a.fsteps = (double*)xs[FS].dev;
    a.status = (int32_t*)xs[SS].dev;
  } else {
    a.state = state; a.v_cur = v_cur; a.h = h; a.l_feet = l_feet; a.v_ref = v_ref; a.reduced = reduced;
    a.gait = gait; a.rot_flag = rot_flag; a.h_rot = h_rot; a.xref = xref; a.fsteps = fsteps; a.status = status;
  }
  HIP_TRY(mpcq::launch_plan(P, a, c->stream));
  if (!dev) return unstage(c, xs, NX);
  if (!(flags & MPCQ_FLAG_ASYNC)) HIP_TRY(hipStreamSynchronize(c->stream));
  return MPCQ_OK;
}

// ---------------------------------------------------------------------------
// Closed-loop session: per-robot state resident in HBM (include/mpcq.h).

}  // extern "C"

struct mpcq_session {
  mpcq_ctx* ctx = nullptr;
  int64_t B = 0;
  mpcq_planner_params pp{};
  void* mem = nullptr;
  void* arr[MPCQ_SV_COUNT] = {};
  size_t bytes[MPCQ_SV_COUNT] = {};
  double* warm_x = nullptr;
  int32_t* plan_status = nullptr;
  int32_t* info = nullptr;
  double* in_state = nullptr;   // staging of host inputs
  double* in_lfeet = nullptr;
  double* in_vref = nullptr;
  int32_t* in_reduced = nullptr;
  int32_t* order = nullptr;  // dispatch order of the next solve (longest previous first)
  bool have_order = false;
  bool use_order = true;  // MPCQ_DISPATCH_ORDER=0 turns it off (A/B timing only; results are identical)
};

namespace {

size_t sv_bytes(int what, int64_t B, int N) {
  const size_t b = (size_t)B;
  switch (what) {
    case MPCQ_SV_F0: return b * 12 * 8;
    case MPCQ_SV_X: return b * 24 * N * 8;
    case MPCQ_SV_X_ROBOT: return b * 12 * N * 8;
    case MPCQ_SV_Q_W: return b * 6 * 8;
    case MPCQ_SV_COST: return b * 13 * 8;
    case MPCQ_SV_XREF: return b * 12 * (N + 1) * 8;
    case MPCQ_SV_FSTEPS: return b * 260 * 8;
    case MPCQ_SV_GAIT: return b * 100 * 8;
    case MPCQ_SV_STATUS: return b * 4;
    case MPCQ_SV_ITERS: return b * 4;
    case MPCQ_SV_RHO: return b * 8;
    case MPCQ_SV_Y: return b * 44 * N * 8;
    case MPCQ_SV_STATE: return b * 12 * 8;
    case MPCQ_SV_L_FEET: return b * 12 * 8;
    case MPCQ_SV_ROT_FLAG: return b * 4;
    case MPCQ_SV_H_ROT: return b * 8;
    case MPCQ_SV_ORDER: return b * 4;
  }
  return 0;
}

}  // namespace

extern "C" {

int mpcq_session_create(mpcq_ctx* c, int64_t B, const mpcq_planner_params* pp, const double* gait0,
                        mpcq_session** out) {
  if (!out) return fail(MPCQ_E_INVALID, "out is NULL");
  *out = nullptr;
  int rc = check_ctx(c, B);
  if (rc) return rc;
  if (B < 1) return fail(MPCQ_E_INVALID, "a session needs batch >= 1");
  const int N = c->N;
  mpcq_session* s = new mpcq_session();
  s->ctx = c;
  s->B = B;
  if (pp) s->pp = *pp;
  else mpcq_default_planner_params(&s->pp);
  // one allocation: the named arrays, then the private ones
  size_t off[MPCQ_SV_COUNT + 8];
  size_t tot = 0;
  auto take = [&](size_t nb) { size_t o = tot; tot += (nb + 255) & ~size_t(255); return o; };
  for (int w = 0; w < MPCQ_SV_COUNT; ++w) { s->bytes[w] = sv_bytes(w, B, N); off[w] = take(s->bytes[w]); }
  const size_t o_wx = take((size_t)B * 24 * N * 8), o_ps = take((size_t)B * 4), o_in = take((size_t)B * 16),
               o_st = take((size_t)B * 96), o_lf = take((size_t)B * 96), o_vr = take((size_t)B * 48),
               o_rd = take((size_t)B * 4);
  DeviceGuard g(c->device);
  if (hipMalloc(&s->mem, tot) != hipSuccess) {
    delete s;
    return fail(MPCQ_E_NOMEM, "hipMalloc(%zu) for the session failed", tot);
  }
  if (hipMemset(s->mem, 0, tot) != hipSuccess) {  // every array defined before the first tick
    (void)hipFree(s->mem);
    delete s;
    return fail(MPCQ_E_DEVICE, "hipMemset of the session failed");
  }
  char* base = (char*)s->mem;
  for (int w = 0; w < MPCQ_SV_COUNT; ++w) s->arr[w] = base + off[w];
  s->warm_x = (double*)(base + o_wx);
  s->plan_status = (int32_t*)(base + o_ps);
  s->info = (int32_t*)(base + o_in);
  s->in_state = (double*)(base + o_st);
  s->in_lfeet = (double*)(base + o_lf);
  s->in_vref = (double*)(base + o_vr);
  s->in_reduced = (int32_t*)(base + o_rd);
  s->order = (int32_t*)s->arr[MPCQ_SV_ORDER];
  {
    const char* e = getenv("MPCQ_DISPATCH_ORDER");
    s->use_order = !(e && e[0] == '0');
  }
  // initial values: the reference objects' constructors
  const size_t hb = sv_bytes(MPCQ_SV_XREF, B, N) > sv_bytes(MPCQ_SV_FSTEPS, B, N) ? sv_bytes(MPCQ_SV_XREF, B, N)
                                                                                  : sv_bytes(MPCQ_SV_FSTEPS, B, N);
  double* h = (double*)malloc(hb > (size_t)B * 100 * 8 ? hb : (size_t)B * 100 * 8);
  int32_t* hi = (int32_t*)malloc((size_t)B * 4);
  if (!h || !hi) { free(h); free(hi); mpcq_session_destroy(s); return fail(MPCQ_E_NOMEM, "host malloc failed"); }
  int err = 0;
  auto put = [&](int w, const void* src) {
    if (!err && hipMemcpy(s->arr[w], src, s->bytes[w], hipMemcpyHostToDevice) != hipSuccess) err = 1;
  };
  if (gait0) {
    put(MPCQ_SV_GAIT, gait0);
  } else {  // create_walking_trot (FootstepPlanner.py:193-214): [1, 7, 1, 7] per 16-step period
    const int half = (int)(0.5 * s->pp.T_gait / s->pp.dt);
    const int per = 2 * half, nper = per > 0 ? N / per : 0;
    if (nper < 1 || nper * per != N || 4 * nper > 19) {
      free(h); free(hi); mpcq_session_destroy(s);
      return fail(MPCQ_E_INVALID, "no walking-trot table for N=%d with T_gait/dt = %d; pass gait0", N, per);
    }
    for (int64_t b = 0; b < B; ++b) {
      double* gt = h + b * 100;
      for (int e = 0; e < 100; ++e) gt[e] = 0.0;
      for (int i = 0; i < nper; ++i) {
        const double d[4] = {1.0, half - 1.0, 1.0, half - 1.0};
        const int m[4][4] = {{1, 1, 1, 1}, {1, 0, 0, 1}, {1, 1, 1, 1}, {0, 1, 1, 0}};
        for (int r = 0; r < 4; ++r) {
          gt[5 * (4 * i + r)] = d[r];
          for (int q = 0; q < 4; ++q) gt[5 * (4 * i + r) + 1 + q] = m[r][q];
        }
      }
    }
    put(MPCQ_SV_GAIT, h);
  }
  for (size_t e = 0; e < (size_t)B * 12 * (N + 1); ++e) h[e] = 0.0;
  put(MPCQ_SV_XREF, h);  // FootstepPlanner.py:58
  for (int64_t b = 0; b < B; ++b) {
    double* q = h + b * 6;  // MPC.py:53-56
    q[0] = 0.0; q[1] = 0.0; q[2] = 0.2027682; q[3] = 0.0; q[4] = 0.0; q[5] = 0.0;
  }
  put(MPCQ_SV_Q_W, h);
  for (int64_t b = 0; b < B; ++b) {  // virtual robot standing at h_ref, feet under the shoulders
    double* st = h + b * 12;
    for (int e = 0; e < 12; ++e) st[e] = 0.0;
    st[2] = s->pp.h_ref;
  }
  put(MPCQ_SV_STATE, h);
  for (int64_t b = 0; b < B; ++b) {
    double* lf = h + b * 12;
    for (int q = 0; q < 4; ++q) { lf[q] = s->pp.shoulders[q]; lf[4 + q] = s->pp.shoulders[4 + q]; lf[8 + q] = 0.0; }
  }
  put(MPCQ_SV_L_FEET, h);
  for (int64_t b = 0; b < B; ++b) h[b] = 0.20;  // FootstepPlanner.py:68
  put(MPCQ_SV_H_ROT, h);
  for (int64_t b = 0; b < B; ++b) h[b] = c->p.rho;
  put(MPCQ_SV_RHO, h);
  for (int64_t b = 0; b < B; ++b) hi[b] = 0;
  put(MPCQ_SV_ROT_FLAG, hi);
  put(MPCQ_SV_STATUS, hi);
  put(MPCQ_SV_ITERS, hi);
  for (int64_t b = 0; b < B; ++b) hi[b] = (int32_t)b;  // a permutation from the start: the identity
  put(MPCQ_SV_ORDER, hi);
  for (size_t e = 0; e < (size_t)B * 260; ++e) h[e] = NAN;
  put(MPCQ_SV_FSTEPS, h);
  free(h);
  free(hi);
  if (err) { mpcq_session_destroy(s); return fail(MPCQ_E_DEVICE, "initialising the session failed"); }
  *out = s;
  return MPCQ_OK;
}

int mpcq_session_destroy(mpcq_session* s) {
  if (!s) return MPCQ_OK;
  if (s->mem) {
    DeviceGuard g(s->ctx->device);
    (void)hipStreamSynchronize(s->ctx->stream);
    (void)hipFree(s->mem);
  }
  delete s;
  return MPCQ_OK;
}

int mpcq_session_tick(mpcq_session* s, int k, const double* state, const double* l_feet, const double* v_ref,
                      const int32_t* reduced, uint32_t flags) {
  if (!s) return fail(MPCQ_E_INVALID, "session is NULL");
  if (!v_ref) return fail(MPCQ_E_INVALID, "v_ref is required");
  if (k < 0) return fail(MPCQ_E_INVALID, "k must be >= 0");
  mpcq_ctx* c = s->ctx;
  DeviceGuard g(c->device);
  const int N = c->N;
  const int64_t B = s->B;
  const bool dev = flags & MPCQ_FLAG_DEVICE_PTRS;
  auto in = [&](const void* src, void* stage_buf, size_t nb) -> const void* {
    if (!src) return nullptr;
    if (dev) return src;
    if (hipMemcpyAsync(stage_buf, src, nb, hipMemcpyHostToDevice, c->stream) != hipSuccess) return nullptr;
    return stage_buf;
  };
  const double* st = state ? (const double*)in(state, s->in_state, (size_t)B * 96) : (const double*)s->arr[MPCQ_SV_STATE];
  const double* lf = l_feet ? (const double*)in(l_feet, s->in_lfeet, (size_t)B * 96) : (const double*)s->arr[MPCQ_SV_L_FEET];
  const double* vr = (const double*)in(v_ref, s->in_vref, (size_t)B * 48);
  const int32_t* rd = reduced ? (const int32_t*)in(reduced, s->in_reduced, (size_t)B * 4) : nullptr;
  if (!st || !lf || !vr || (reduced && !rd)) return fail(MPCQ_E_DEVICE, "staging the tick inputs failed");
  // the virtual robot's state lives in buffers the retrieve kernel rewrites:
  // this tick reads a copy
  if (!state) {
    HIP_TRY(hipMemcpyAsync(s->in_state, st, (size_t)B * 96, hipMemcpyDeviceToDevice, c->stream));
    st = s->in_state;
  }
  if (!l_feet) {
    HIP_TRY(hipMemcpyAsync(s->in_lfeet, lf, (size_t)B * 96, hipMemcpyDeviceToDevice, c->stream));
    lf = s->in_lfeet;
  }
  // 1. planner (processing.py:80-89, 131)
  mpcq::PlanArgs pa{};
  pa.batch = B;
  pa.N = N;
  pa.k = k;
  pa.state = st;
  pa.l_feet = lf;
  pa.v_ref = vr;
  pa.reduced = rd;
  pa.gait = (double*)s->arr[MPCQ_SV_GAIT];
  pa.rot_flag = (int32_t*)s->arr[MPCQ_SV_ROT_FLAG];
  pa.h_rot = (double*)s->arr[MPCQ_SV_H_ROT];
  pa.xref = (double*)s->arr[MPCQ_SV_XREF];
  pa.fsteps = (double*)s->arr[MPCQ_SV_FSTEPS];
  pa.status = s->plan_status;
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  if (k == 0) {  // update_fsteps(0, ...): no roll
    pa.ops = MPCQ_PLAN_FOOTSTEPS;
    HIP_TRY(mpcq::launch_plan(s->pp, pa, c->stream));
  }
  pa.ops = MPCQ_PLAN_TICK;
  HIP_TRY(mpcq::launch_plan(s->pp, pa, c->stream));
  HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  c->have_form = true;
  // 2. MPC.run: formulation + OSQP solve (warm from the previous tick when k > 0)
  mpcq::LaunchArgs la{};
  la.batch = B;
  la.mode = k == 0 ? MPCQ_MODE_SETUP : MPCQ_MODE_UPDATE;
  la.xref = (const double*)s->arr[MPCQ_SV_XREF];
  la.fsteps = (const double*)s->arr[MPCQ_SV_FSTEPS];
  if (k > 0) {
    la.warm_x = s->warm_x;
    la.warm_y = (const double*)s->arr[MPCQ_SV_Y];
    la.rho_in = (const double*)s->arr[MPCQ_SV_RHO];
  }
  la.f0 = (double*)s->arr[MPCQ_SV_F0];
  la.x = (double*)s->arr[MPCQ_SV_X];
  la.y = (double*)s->arr[MPCQ_SV_Y];
  la.status = (int32_t*)s->arr[MPCQ_SV_STATUS];
  la.iters = (int32_t*)s->arr[MPCQ_SV_ITERS];
  la.rho_out = (double*)s->arr[MPCQ_SV_RHO];
  la.info = s->info;
  la.stamps = c->stamps;
  // longest-first by the previous tick's iteration counts (a tick k == 0 restarts cold)
  if (k == 0) s->have_order = false;
  la.order = s->have_order && s->use_order ? s->order : nullptr;
  {
    const int wrc = ensure_work(c, B, &la.work);
    if (wrc) return wrc;
  }
  HIP_TRY(hipEventRecord(c->ev[2], c->stream));
  HIP_TRY(mpcq::launch_solve(N, true, c->p, la, c->stream));
  HIP_TRY(hipEventRecord(c->ev[3], c->stream));
  c->have_solve = true;
  // 3. retrieve_result, q_w, Logger cost, next warm start, virtual robot
  mpcq::SessionArgs ra{};
  ra.batch = B;
  ra.x = (const double*)s->arr[MPCQ_SV_X];
  ra.xref = (const double*)s->arr[MPCQ_SV_XREF];
  ra.fsteps = (const double*)s->arr[MPCQ_SV_FSTEPS];
  ra.gait = (const double*)s->arr[MPCQ_SV_GAIT];
  ra.status = (int32_t*)s->arr[MPCQ_SV_STATUS];
  ra.plan_status = s->plan_status;
  ra.x_robot = (double*)s->arr[MPCQ_SV_X_ROBOT];
  ra.warm_x = s->warm_x;
  ra.y = (double*)s->arr[MPCQ_SV_Y];
  ra.rho = (double*)s->arr[MPCQ_SV_RHO];
  ra.rho0 = c->p.rho;
  ra.cost = (double*)s->arr[MPCQ_SV_COST];
  ra.q_w = (double*)s->arr[MPCQ_SV_Q_W];
  ra.next_state = (double*)s->arr[MPCQ_SV_STATE];
  ra.next_l_feet = (double*)s->arr[MPCQ_SV_L_FEET];
  for (int i = 0; i < 12; ++i) ra.state_weights[i] = c->p.state_weights[i];
  ra.force_weight = c->p.force_weight;
  for (int i = 0; i < 8; ++i) ra.shoulders[i] = s->pp.shoulders[i];
  HIP_TRY(mpcq::launch_retrieve(N, ra, c->stream));
  HIP_TRY(mpcq::launch_order((const int32_t*)s->arr[MPCQ_SV_ITERS], B, s->order, c->stream));
  s->have_order = true;
  // host inputs are staged in buffers the next tick reuses: host calls block
  if (!(flags & MPCQ_FLAG_ASYNC) || !dev) HIP_TRY(hipStreamSynchronize(c->stream));
  return MPCQ_OK;
}

int mpcq_session_read(mpcq_session* s, int what, void* dst, uint32_t flags) {
  if (!s || !dst) return fail(MPCQ_E_INVALID, "NULL argument");
  if (what < 0 || what >= MPCQ_SV_COUNT) return fail(MPCQ_E_INVALID, "unknown session array %d", what);
  DeviceGuard g(s->ctx->device);
  const hipMemcpyKind kind = (flags & MPCQ_FLAG_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  HIP_TRY(hipMemcpyAsync(dst, s->arr[what], s->bytes[what], kind, s->ctx->stream));
  HIP_TRY(hipStreamSynchronize(s->ctx->stream));
  return MPCQ_OK;
}

int mpcq_session_write(mpcq_session* s, int what, const void* src, uint32_t flags) {
  if (!s || !src) return fail(MPCQ_E_INVALID, "NULL argument");
  if (what < 0 || what >= MPCQ_SV_COUNT) return fail(MPCQ_E_INVALID, "unknown session array %d", what);
  // the engine indexes robots through the order: only order_kernel writes it
  if (what == MPCQ_SV_ORDER) return fail(MPCQ_E_INVALID, "MPCQ_SV_ORDER is read-only");
  DeviceGuard g(s->ctx->device);
  const hipMemcpyKind kind = (flags & MPCQ_FLAG_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIP_TRY(hipMemcpyAsync(s->arr[what], src, s->bytes[what], kind, s->ctx->stream));
  HIP_TRY(hipStreamSynchronize(s->ctx->stream));
  return MPCQ_OK;
}

int mpcq_session_device_ptr(mpcq_session* s, int what, void** out) {
  if (!s || !out) return fail(MPCQ_E_INVALID, "NULL argument");
  if (what < 0 || what >= MPCQ_SV_COUNT) return fail(MPCQ_E_INVALID, "unknown session array %d", what);
  *out = s->arr[what];
  return MPCQ_OK;
}

int mpcq_debug_set_stamps(mpcq_ctx* c, void* buf) {
  if (!c) return fail(MPCQ_E_INVALID, "ctx is NULL");
  c->stamps = (uint64_t*)buf;
  return MPCQ_OK;
}

}  // extern "C"
