// api.hip — error plumbing and version of the C-ABI (include/unet_hip.h).
#include "common.h"
#include <stdio.h>

namespace unet {
static thread_local char g_err[512] = "";
void set_error(const char* msg) { snprintf(g_err, sizeof(g_err), "%s", msg); }
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}
}  // namespace unet

extern "C" {
const char* unet_last_error(void) { return unet::g_err; }
int unet_version(void) { return UNET_ABI_VERSION; }
}
