// mpcq_dispatch.cpp — horizon dispatch of the engine.  mpcq_engine.hip is
// compiled once per horizon (Makefile: -DMPCQ_ENGINE_N=N); each unit exports
// engine_launch_n<N>, and this file maps a context's N onto it.
//
// Horizons compiled in: every N from 4 to 64 (MPC.py takes any n_steps,
// MPC.py:22-26; FootstepPlanner.py:55 gives n_periods * T_gait / dt).  A wave64
// holds four 16-lane stage rows; N that is not a multiple of 4 runs the rows past
// N as copies of stage N-1 (kRows in mpcq_engine.hip).  Up to 16 stages two
// instances share a CU, up to 32 one (LDS, checked by static_asserts in
// mpcq_engine.hip); beyond 32, S^{-1} and R^{-1} Q live in a per-instance
// global workspace (work_doubles), beyond 49 the scaled constraint values too (kAbG).
#include "mpcq_internal.h"

namespace mpcq {

#define MPCQ_DECL(NN) \
  hipError_t engine_launch_n##NN(bool fused, bool solve, const mpcq_params& p, const LaunchArgs& a, hipStream_t s);
MPCQ_HORIZONS(MPCQ_DECL)
#undef MPCQ_DECL

bool horizon_supported(int N) {
#define MPCQ_CASE(NN) case NN:
  switch (N) {
    MPCQ_HORIZONS(MPCQ_CASE) return true;
    default: return false;
  }
#undef MPCQ_CASE
}

int supported_horizons(int32_t* out, int cap) {
  int n = 0;
#define MPCQ_LIST(NN) { if (n < cap) out[n] = NN; ++n; }
  MPCQ_HORIZONS(MPCQ_LIST)
#undef MPCQ_LIST
  return n;
}

static hipError_t launch_any(int N, bool fused, bool solve, const mpcq_params& p, const LaunchArgs& a,
                             hipStream_t s) {
  if (a.batch <= 0) return hipSuccess;
#define MPCQ_CASE(NN) case NN: return engine_launch_n##NN(fused, solve, p, a, s);
  switch (N) {
    MPCQ_HORIZONS(MPCQ_CASE)
    default: return hipErrorInvalidValue;
  }
#undef MPCQ_CASE
}

hipError_t launch_formulate(int N, const mpcq_params& p, const LaunchArgs& a, hipStream_t s) {
  return launch_any(N, true, false, p, a, s);
}

hipError_t launch_solve(int N, bool fused, const mpcq_params& p, const LaunchArgs& a, hipStream_t s) {
  return launch_any(N, fused, true, p, a, s);
}

}  // namespace mpcq
