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
};

// Launchers (mpcq_kernels.hip).  Return hipError_t.
hipError_t launch_formulate(int N, const mpcq_params& p, const LaunchArgs& a, hipStream_t s);
hipError_t launch_solve(int N, bool fused, const mpcq_params& p, const LaunchArgs& a, hipStream_t s);
bool horizon_supported(int N);
int supported_horizons(int32_t* out, int cap);

}  // namespace mpcq
