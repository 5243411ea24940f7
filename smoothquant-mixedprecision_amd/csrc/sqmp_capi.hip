// Library identity and status strings of the C ABI (include/sqmp_w4a4.h).
#include "sqmp_common.h"

extern "C" const char* sqmp_version(void) {
  return "sqmp_w4a4 0.6.1 (gfx950; W4A4 mixed-precision linear, smoothquant-mixedprecision)";
}

extern "C" const char* sqmp_status_string(int status) {
  switch (status) {
    case SQMP_OK: return "ok";
    case SQMP_EINVAL: return "invalid argument";
    case SQMP_EUNSUPPORTED: return "unsupported configuration";
    case SQMP_EHIP: return "HIP runtime error";
    case SQMP_EWORKSPACE: return "workspace missing or too small";
    default: return "unknown status";
  }
}
