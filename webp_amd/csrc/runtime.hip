// runtime.hip -- library-wide C-ABI entry points: error reporting, version,
// device check.  There is deliberately no CPU fallback anywhere in
// libwebpgpu.so: a missing / non-gfx950 device is an error.
#include <string.h>

#include <mutex>

#include "wg_common.h"

namespace wg {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

int stream_device(hipStream_t s, int* dev) {
  hipDevice_t d = 0;
  // the null stream is the current device's (hipStreamGetDevice says so too)
  if ((s ? hipStreamGetDevice(s, &d) : hipGetDevice(&d)) != hipSuccess || d < 0 || d >= 64) {
    set_error("stream_device: cannot tell the stream's device");
    return WG_EHIP;
  }
  *dev = d;
  return WG_OK;
}

namespace {
std::mutex g_diag_mu;
int* g_diag_blocks[64] = {nullptr};
// per device and kernel family: the count of timed-out waits the status
// entry points have already reported (diag[0] is cumulative on the device)
int g_diag_reported[64][4] = {{0}};
}  // namespace

// one 64-int block per device -- the device the stream `s` belongs to --
// zeroed once on that stream (a queue already in use: no new hardware queue
// is created for it)
int* diag_words(hipStream_t s) {
  int dev = 0;
  if (stream_device(s, &dev) != WG_OK) return nullptr;
  std::lock_guard<std::mutex> lock(g_diag_mu);
  int*(&blocks)[64] = g_diag_blocks;
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

int take_new_timeouts(hipStream_t s, int family, int total) {
  int dev = 0;
  if (stream_device(s, &dev) != WG_OK) return total;
  std::lock_guard<std::mutex> lock(g_diag_mu);
  int& seen = g_diag_reported[dev][(family / 16) & 3];
  const int fresh = total - seen;
  seen = total;
  return fresh > 0 ? fresh : 0;
}

namespace {
__global__ void k_inject_timeout(int* diag) { note_timeout(diag, -1, -1, -1, -1, -1, -1); }
}  // namespace
}  // namespace wg

extern "C" int wg_debug_inject_timeout(int32_t family, void* stream) {
  WG_REQUIRE(family == wg::DIAG_ENCODE || family == wg::DIAG_DECODE || family == wg::DIAG_VP8L_INVERSE ||
             family == wg::DIAG_ALPHA);
  hipStream_t s = wg::as_stream(stream);
  int* diag = wg::diag_words(s);
  if (!diag) return WG_EHIP;
  hipLaunchKernelGGL(wg::k_inject_timeout, dim3(1), dim3(1), 0, s, diag + family);
  return wg::check_launch("k_inject_timeout");
}

extern "C" const char* wg_last_error(void) { return wg::g_last_error.c_str(); }

extern "C" int wg_version(void) { return WG_ABI_VERSION; }

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
