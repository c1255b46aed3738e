// mpcq_build.cpp -- the library's build stamp (include/mpcq.h mpcq_build_info).
// The Makefile hashes the HIP sources (csrc/*.hip in name order) and passes the first
// 16 hex digits as MPCQ_SRC_SHA; profiles record the stamp of the build they measured.
#include "../../include/mpcq.h"

#ifndef MPCQ_SRC_SHA
#define MPCQ_SRC_SHA "unknown"
#endif
#ifndef MPCQ_ARCH
#define MPCQ_ARCH "unknown"
#endif

extern "C" const char* mpcq_build_info(void) { return "src_sha256=" MPCQ_SRC_SHA " arch=" MPCQ_ARCH; }
