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

// The device a stream belongs to (the current device for the null stream).
int stream_device(hipStream_t s, int* dev);

// Timed-out dependency waits of the persistent kernels, per device (the
// device of stream s): a zeroed, never-reset block of 16 ints per kernel
// family (DIAG_ENCODE ...): [0] timed-out waits of every launch since the
// library loaded, [1] set once the first one is recorded, [2..7] its
// coordinates (kernel-specific).  Returns nullptr (error set) if the block
// cannot be made.
enum { DIAG_ENCODE = 0, DIAG_DECODE = 16, DIAG_VP8L_INVERSE = 32, DIAG_ALPHA = 48 };
int* diag_words(hipStream_t s);
// Of the cumulative count `total` of a family on s's device, how many no
// status call has reported yet; marks them reported.
int take_new_timeouts(hipStream_t s, int family, int total);

// lane-0 call on a timed-out wait: counts it and records the first one
// s_memrealtime for the start of a bounded wait, waited for at once.  The
// wait's slow path reads it; left outstanding, it reaches the join with the
// fast path, where the compiler then puts an lgkmcnt(0) -- which waits for
// every LDS read in flight too -- before the first reuse of its SGPRs, on
// every pass of the fast path (round 6: one a step in k_vp8l_inverse's walk).
// 0xC07F = lgkmcnt(0), vmcnt / expcnt unconstrained; the builtin, unlike
// inline asm, is seen by the compiler's wait bookkeeping.
__device__ __forceinline__ uint64_t wait_clock() {
  const uint64_t t = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  return t;
}

__device__ inline void note_timeout(int* diag, int c2, int c3, int c4, int c5, int c6, int c7) {
  __hip_atomic_fetch_add(&diag[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int z = 0;
  if (__hip_atomic_compare_exchange_strong(&diag[1], &z, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)) {
    const int v[6] = {c2, c3, c4, c5, c6, c7};
#pragma unroll
    for (int k = 0; k < 6; k++) __hip_atomic_store(&diag[2 + k], v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The status entry points of the persistent kernels: `flag` is the launch's
// own timeout word in its work buffer (cleared by each launch), `diag` the
// device's cumulative record of timed-out waits of every launch of that
// kernel family (diag_words).  A timeout in any launch -- not only the last
// one on `work` -- is reported by the first status call after it, and only
// by that one: once reported, later clean launches return WG_OK again (a
// long-lived host survives one transient stall).  `fields` names diag[2..7].
// Synchronises `s`.
inline int wait_status(const int* flag, int family, hipStream_t s, const char* what, const char* fields) {
  int* diag = diag_words(s);
  if (!diag) return WG_EHIP;
  int f = 0, d[8] = {0};
  if (hipMemcpyAsync(&f, flag, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(d, diag + family, sizeof(d), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return check_launch(what);
  const int fresh = take_new_timeouts(s, family, d[0]);
  if (f || fresh) {
    std::string m = std::string(what) + ": a dependency wait timed out (output invalid)" +
                    (f ? "" : " in an earlier launch") + "; " + std::to_string(fresh) + " new timed-out waits (" +
                    std::to_string(d[0]) + " since the library loaded)";
    if (d[1]) {
      m += ", the first at (" + std::string(fields) + ") =";
      for (int k = 2; k < 8; k++) m += " " + std::to_string(d[k]);
    }
    set_error(m);
    return WG_EHIP;
  }
  return WG_OK;
}

}  // namespace wg

#define WG_REQUIRE(cond)                   \
  do {                                     \
    if (!(cond)) return wg::invalid(#cond); \
  } while (0)
