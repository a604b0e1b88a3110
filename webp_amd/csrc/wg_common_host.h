// wg_common_host.h -- error / argument helpers for host-only (no HIP) C-ABI
// translation units; the same contract as wg_common.h.
#pragma once
#include <stdint.h>

#include <string>

#include "../../include/webpgpu.h"

namespace wg {
void set_error(const std::string& msg);
inline int invalid(const char* what) {
  set_error(std::string("invalid argument: ") + what);
  return WG_EINVAL;
}
}  // namespace wg

#define WG_REQUIRE(cond)                   \
  do {                                     \
    if (!(cond)) return wg::invalid(#cond); \
  } while (0)
