// wg_instr.h -- every measurement / diagnostic hook of the kernels, in one
// place.  The product build defines none of the switches below, and every
// hook then compiles to nothing (WG_REP_BEGIN / END to a one-trip loop the
// compiler removes); the kernels carry no other build switches.
//
//   -DWG_BOUNDS          WG_IN(p, bytes, base, size, flag): the global access
//                        at that site checked against its buffer's extent; one
//                        outside it is skipped and ORs 4 into *flag (the
//                        launch's status word), tools/gpu_bounds_suite.sh
//   -DWG_STAMPS          per-phase cycle stamps: the decoder's STAMP(k)
//                        (wg_debug_phases), the encoder's ESTAMP / SSTAMP /
//                        CSTAMP / DSTAMP (wg_debug_enc_phases)
//   -DWG_ROWTIMES        the encoder's per-row timeline (wg_debug_enc_rows,
//                        tools/enc_timeline.py)
//   -DWG_EXP_REP_<P>=N   an encoder phase run N times per macroblock: P = RD
//                        (I16 + UV RD), I4 (the whole I4 RD), PRE (value table
//                        + pre-screen), CAND (candidates' prediction +
//                        FTransform), PREP (trellis records), DP (the trellis
//                        DP), FIN (final residuals).  Each phase is idempotent,
//                        so the outputs stay bit-exact and a counter of the
//                        build minus the product's is that phase's own share
//                        (tools/gpu_enc_phase_sq.sh)
//   -DWG_DEC_SKIPW=mask  bit k drops k_decode_bands' store site k (WRITE_SIZE
//                        per site, tools/gpu_dec_write_sites.sh; the output is
//                        then wrong, the control flow unchanged)
//   -DWG_TIMELINES       per-wave timelines of the dependency walks: the VP8L
//                        inverse's bands (tools/inv_timeline.py) and SharpYUV's
//                        (image, iteration, band) waves (tools/sharp_timeline.py)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// ---- WG_BOUNDS ----
// WG_CHK(p, bytes, base, size, "site"): the access of `bytes` at p must lie in
// [base, base + size) -- the buffer's extent implied by the entry point's
// shape arguments; one outside it is skipped and printed (device printf, one
// line per lane: tools/gpu_bounds_suite.sh greps the log for "WG_BOUNDS").
// WG_IN also ORs 4 into the launch's status word (*flag).
#ifdef WG_BOUNDS
__device__ __forceinline__ bool wg_chk(const void* p, int bytes, const void* base, int64_t size, const char* site) {
  const int64_t o = static_cast<const char*>(p) - static_cast<const char*>(base);
  const bool ok = o >= 0 && o + bytes <= size;
  if (!ok)
    printf("WG_BOUNDS %s: bytes [%lld, %lld) of a %lld-byte buffer, block %d thread %d\n", site, (long long)o,
           (long long)(o + bytes), (long long)size, (int)blockIdx.x, (int)threadIdx.x);
  return ok;
}
__device__ __forceinline__ bool wg_in_buf(const void* p, int bytes, const void* base, int64_t size, int* flag) {
  const bool ok = wg_chk(p, bytes, base, size, "k_decode_bands");
  if (!ok) __hip_atomic_fetch_or(flag, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ok;
}
#define WG_CHK(p, bytes, base, size, site) wg_chk((p), (bytes), (base), (size), (site))
#define WG_IN(p, bytes, base, size, flag) wg_in_buf((p), (bytes), (base), (size), (flag))
#else
#define WG_CHK(p, bytes, base, size, site) true
#define WG_IN(p, bytes, base, size, flag) true
#endif

// ---- WG_DEC_SKIPW ----
#ifndef WG_DEC_SKIPW
#define WG_DEC_SKIPW 0
#endif
#define DEC_SITE(bit) ((WG_DEC_SKIPW & (bit)) == 0)

// ---- WG_STAMPS / WG_ROWTIMES / WG_TIMELINES: code present only in those builds ----
#ifdef WG_STAMPS
#define WG_IF_STAMPS(...) __VA_ARGS__
#else
#define WG_IF_STAMPS(...)
#endif
#ifdef WG_ROWTIMES
#define WG_IF_ROWTIMES(...) __VA_ARGS__
#else
#define WG_IF_ROWTIMES(...)
#endif
#ifdef WG_TIMELINES
#define WG_IF_TIMELINES(...) __VA_ARGS__
#else
#define WG_IF_TIMELINES(...)
#endif

#define WG_STAMP_NOW(ts_)                                                        \
  __builtin_amdgcn_sched_barrier(0);                                             \
  unsigned long long ts_;                                                        \
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts_)::"memory");  \
  __builtin_amdgcn_sched_barrier(0)

#ifdef WG_STAMPS
// decoder: cycles per phase, summed over macroblocks (g_phase, wg_debug_phases)
#define STAMP_DECL unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0
#define STAMP(k)                                  \
  do {                                            \
    WG_STAMP_NOW(ts_);                            \
    if ((k) > 0) st_acc[(k)-1] += ts_ - st_prev;  \
    st_prev = ts_;                                \
  } while (0)
#define STAMP_FLUSH()                                                      \
  do {                                                                     \
    if (lane == 0)                                                         \
      for (int k_ = 0; k_ < 10; k_++) atomicAdd(&g_phase[k_], st_acc[k_]); \
  } while (0)
// encoder: phases into st_acc[k - 1], sub-phases [8 + k], candidate-internal
// [12 + k], the I4 trellis DP alone [7] (g_enc_phase, wg_debug_enc_phases)
#define ESTAMP_DECL \
  unsigned long long st_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0, sub_prev = 0, cst_prev = 0, dst_prev = 0
#define ESTAMP(k)                                 \
  do {                                            \
    WG_STAMP_NOW(ts_);                            \
    if ((k) > 0) st_acc[(k)-1] += ts_ - st_prev;  \
    st_prev = ts_;                                \
  } while (0)
#define ESTAMP_FLUSH()                                                          \
  do {                                                                          \
    if (lane == 0)                                                              \
      for (int k_ = 0; k_ < 16; k_++) atomicAdd(&g_enc_phase[k_], st_acc[k_]); \
  } while (0)
#define SSTAMP(k)                                      \
  do {                                                 \
    WG_STAMP_NOW(ts_);                                 \
    if ((k) >= 0) st_acc[8 + (k)] += ts_ - sub_prev;   \
    sub_prev = ts_;                                    \
  } while (0)
#define CSTAMP(k)                                      \
  do {                                                 \
    WG_STAMP_NOW(ts_);                                 \
    if ((k) >= 0) st_acc[12 + (k)] += ts_ - cst_prev;  \
    cst_prev = ts_;                                    \
  } while (0)
#define DSTAMP(k)                                 \
  do {                                            \
    WG_STAMP_NOW(ts_);                            \
    if ((k) >= 0) st_acc[7] += ts_ - dst_prev;    \
    dst_prev = ts_;                               \
  } while (0)
#else
#define STAMP_DECL int st_unused_ = 0
#define STAMP(k) (void)st_unused_
#define STAMP_FLUSH() (void)st_unused_
#define ESTAMP_DECL int st_unused_ = 0
#define ESTAMP(k) (void)st_unused_
#define ESTAMP_FLUSH() (void)st_unused_
#define SSTAMP(k) (void)0
#define CSTAMP(k) (void)0
#define DSTAMP(k) (void)0
#endif

// ---- WG_EXP_REP_<P> ----
#ifndef WG_EXP_REP_RD
#define WG_EXP_REP_RD 1
#endif
#ifndef WG_EXP_REP_I4
#define WG_EXP_REP_I4 1
#endif
#ifndef WG_EXP_REP_PRE
#define WG_EXP_REP_PRE 1
#endif
#ifndef WG_EXP_REP_CAND
#define WG_EXP_REP_CAND 1
#endif
#ifndef WG_EXP_REP_PREP
#define WG_EXP_REP_PREP 1
#endif
#ifndef WG_EXP_REP_DP
#define WG_EXP_REP_DP 1
#endif
#ifndef WG_EXP_REP_FIN
#define WG_EXP_REP_FIN 1
#endif
#define WG_REP_BEGIN(P) for (int rep_ = 0; rep_ < WG_EXP_REP_##P; rep_++) {
#define WG_REP_END }
