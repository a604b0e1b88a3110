// wg_common.h -- host-side helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/webpgpu.h"

namespace wg {

void set_error(const std::string& msg);

// Checks the last launch; records the HIP error string on failure.
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return WG_EHIP;
  }
  return WG_OK;
}

inline int invalid(const char* what) {
  set_error(std::string("invalid argument: ") + what);
  return WG_EINVAL;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace wg

#define WG_REQUIRE(cond)                   \
  do {                                     \
    if (!(cond)) return wg::invalid(#cond); \
  } while (0)
