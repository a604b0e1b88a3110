/*
 * dsp_filter.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates internal/dsp/filter.go (the decoder's local copies in
 * internal/lossy/decode_frame.go:360-558 compute the same functions).
 * The clip tables (cliptables.go:9-21) are exact clamps on their domains.
 */
#include "oracle.h"

static inline int sclip1(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); } /* [-893,892] */
static inline int sclip2(int v) { return v < -16 ? -16 : (v > 15 ? 15 : v); }     /* [-112,112] */
static inline uint8_t clip1(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
static inline int iabs(int v) { return v < 0 ? -v : v; }

/* needsFilter :13 (t is already 2*thresh+1) */
static inline int needs_filter(const uint8_t* p, int off, int step, int t) {
  int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  return 4 * iabs(p0 - q0) + iabs(p1 - q1) <= t;
}
/* needsFilter2 :18 */
static inline int needs_filter2(const uint8_t* p, int off, int step, int t, int it) {
  int p3 = p[off - 4 * step], p2 = p[off - 3 * step], p1 = p[off - 2 * step], p0 = p[off - step];
  int q0 = p[off], q1 = p[off + step], q2 = p[off + 2 * step], q3 = p[off + 3 * step];
  if (4 * iabs(p0 - q0) + iabs(p1 - q1) > t) return 0;
  return iabs(p3 - p2) <= it && iabs(p2 - p1) <= it && iabs(p1 - p0) <= it &&
         iabs(q3 - q2) <= it && iabs(q2 - q1) <= it && iabs(q1 - q0) <= it;
}
/* hev :31 */
static inline int hev(const uint8_t* p, int off, int step, int t) {
  int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  return iabs(p1 - p0) > t || iabs(q1 - q0) > t;
}
/* doFilter2 :37 */
static inline void do_filter2(uint8_t* p, int off, int step) {
  int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  int a = 3 * (q0 - p0) + sclip1(p1 - q1);
  int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
  p[off - step] = clip1(p0 + a2);
  p[off] = clip1(q0 - a1);
}
/* doFilter4 :52 */
static inline void do_filter4(uint8_t* p, int off, int step) {
  int p1 = p[off - 2 * step], p0 = p[off - step], q0 = p[off], q1 = p[off + step];
  int a = 3 * (q0 - p0);
  int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
  p[off - 2 * step] = clip1(p1 + a3);
  p[off - step] = clip1(p0 + a2);
  p[off] = clip1(q0 - a1);
  p[off + step] = clip1(q1 - a3);
}
/* doFilter6 :69 */
static inline void do_filter6(uint8_t* p, int off, int step) {
  int p2 = p[off - 3 * step], p1 = p[off - 2 * step], p0 = p[off - step];
  int q0 = p[off], q1 = p[off + step], q2 = p[off + 2 * step];
  int a = sclip1(3 * (q0 - p0) + sclip1(p1 - q1));
  int a1 = (27 * a + 63) >> 7, a2 = (18 * a + 63) >> 7, a3 = (9 * a + 63) >> 7;
  p[off - 3 * step] = clip1(p2 + a3);
  p[off - 2 * step] = clip1(p1 + a2);
  p[off - step] = clip1(p0 + a1);
  p[off] = clip1(q0 - a1);
  p[off + step] = clip1(q1 - a2);
  p[off + 2 * step] = clip1(q2 - a3);
}

/* simple filter across one edge; hstride = step across the edge, vstride = along it */
static void simple_edge(uint8_t* p, int base, int hstride, int vstride, int thresh) {
  int t2 = 2 * thresh + 1;
  for (int i = 0; i < 16; i++) {
    int off = base + i * vstride;
    if (needs_filter(p, off, hstride, t2)) do_filter2(p, off, hstride);
  }
}
void or_simple_vfilter16(uint8_t* p, int base, int stride, int thresh) { simple_edge(p, base, stride, 1, thresh); }
void or_simple_hfilter16(uint8_t* p, int base, int stride, int thresh) { simple_edge(p, base, 1, stride, thresh); }
void or_simple_vfilter16i(uint8_t* p, int base, int stride, int thresh) {
  for (int k = 1; k <= 3; k++) or_simple_vfilter16(p, base + 4 * k * stride, stride, thresh);
}
void or_simple_hfilter16i(uint8_t* p, int base, int stride, int thresh) {
  for (int k = 1; k <= 3; k++) or_simple_hfilter16(p, base + 4 * k, stride, thresh);
}

/* filterLoop26 :144 (mb edge, 6-tap) and filterLoop24 :169 (inner, 4-tap) */
static void filter_loop(uint8_t* p, int base, int hstride, int vstride, int size, int thresh,
                        int ithresh, int hev_t, int inner) {
  int t2 = 2 * thresh + 1;
  for (int i = 0; i < size; i++) {
    int off = base + i * vstride;
    if (!needs_filter2(p, off, hstride, t2, ithresh)) continue;
    if (hev(p, off, hstride, hev_t)) do_filter2(p, off, hstride);
    else if (inner) do_filter4(p, off, hstride);
    else do_filter6(p, off, hstride);
  }
}

void or_vfilter16(uint8_t* p, int base, int stride, int t, int it, int h) { filter_loop(p, base, stride, 1, 16, t, it, h, 0); }
void or_hfilter16(uint8_t* p, int base, int stride, int t, int it, int h) { filter_loop(p, base, 1, stride, 16, t, it, h, 0); }
void or_vfilter16i(uint8_t* p, int base, int stride, int t, int it, int h) {
  for (int k = 1; k <= 3; k++) filter_loop(p, base + 4 * k * stride, stride, 1, 16, t, it, h, 1);
}
void or_hfilter16i(uint8_t* p, int base, int stride, int t, int it, int h) {
  for (int k = 1; k <= 3; k++) filter_loop(p, base + 4 * k, 1, stride, 16, t, it, h, 1);
}
void or_vfilter8(uint8_t* u, uint8_t* v, int ub, int vb, int stride, int t, int it, int h) {
  filter_loop(u, ub, stride, 1, 8, t, it, h, 0);
  filter_loop(v, vb, stride, 1, 8, t, it, h, 0);
}
void or_hfilter8(uint8_t* u, uint8_t* v, int ub, int vb, int stride, int t, int it, int h) {
  filter_loop(u, ub, 1, stride, 8, t, it, h, 0);
  filter_loop(v, vb, 1, stride, 8, t, it, h, 0);
}
void or_vfilter8i(uint8_t* u, uint8_t* v, int ub, int vb, int stride, int t, int it, int h) {
  filter_loop(u, ub + 4 * stride, stride, 1, 8, t, it, h, 1);
  filter_loop(v, vb + 4 * stride, stride, 1, 8, t, it, h, 1);
}
void or_hfilter8i(uint8_t* u, uint8_t* v, int ub, int vb, int stride, int t, int it, int h) {
  filter_loop(u, ub + 4, 1, stride, 8, t, it, h, 1);
  filter_loop(v, vb + 4, 1, stride, 8, t, it, h, 1);
}
