// runtime.hip -- library-wide C-ABI entry points: error reporting, version,
// device check.  There is deliberately no CPU fallback anywhere in
// libwebpgpu.so: a missing / non-gfx950 device is an error.
#include <string.h>

#include <mutex>

#include "wg_common.h"

namespace wg {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// one 64-int block per device, zeroed once on the caller's stream (a queue
// already in use: no new hardware queue is created for it)
int* diag_words(hipStream_t s) {
  static std::mutex mu;
  static int* blocks[64] = {nullptr};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("diag_words: hipGetDevice");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(mu);
  if (!blocks[dev]) {
    int* p = nullptr;
    if (hipMalloc(&p, 64 * sizeof(int)) != hipSuccess || hipMemsetAsync(p, 0, 64 * sizeof(int), s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      set_error("diag_words: allocation failed");
      return nullptr;
    }
    blocks[dev] = p;
  }
  return blocks[dev];
}
}  // namespace wg

extern "C" const char* wg_last_error(void) { return wg::g_last_error.c_str(); }

extern "C" int wg_version(void) { return 1; }

extern "C" int wg_device_check(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    wg::set_error("hipGetDevice failed: no HIP device");
    return WG_ENODEV;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    wg::set_error("hipGetDeviceProperties failed");
    return WG_ENODEV;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    wg::set_error(std::string("unsupported device arch: ") + prop.gcnArchName + " (built for gfx950)");
    return WG_ENODEV;
  }
  return WG_OK;
}
