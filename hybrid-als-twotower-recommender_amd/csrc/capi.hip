// Error plumbing and version of the C-ABI (include/hrec.h).
#include <stdarg.h>

#include <mutex>
#include <set>
#include <utility>

#include "common.h"

namespace hrec {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return HREC_E_LAUNCH;
  }
  return HREC_OK;
}

// Kernels that take more than 64 KiB of dynamic LDS need the attribute raised
// once per (device, kernel): it is set through the current device, so a
// process that drives several GPUs (hipSetDevice) raises it on each.
bool allow_max_lds_ptr(const void* kfn) {
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({dev, kfn})) return true;
  // the CU's 160 KiB less the kernel's static LDS (the attribute bounds the sum)
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, kfn) != hipSuccess) return false;
  const int dyn = 160 * 1024 - (int)fa.sharedSizeBytes;
  if (hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, dyn) != hipSuccess) return false;
  done.insert({dev, kfn});
  return true;
}

}  // namespace hrec

extern "C" int hrec_abi_version(void) { return HREC_ABI_VERSION; }

extern "C" const char* hrec_last_error(void) { return hrec::g_last_error; }
