// C-ABI error plumbing shared by all entry points.
#include <stdarg.h>

#include "trk_common.h"

namespace trk {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return TRK_ELAUNCH;
  }
  return TRK_OK;
}

}  // namespace trk

extern "C" int trk_abi_version(void) { return TRK_ABI_VERSION; }
extern "C" const char* trk_last_error(void) { return trk::g_err; }
