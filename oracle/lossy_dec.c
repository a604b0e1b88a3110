/*
 * lossy_dec.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates the VP8 decoder's DSP driver loops:
 *   reconstructRow        internal/lossy/decode_frame.go:83-218
 *   doTransform / UV      internal/lossy/decode_frame.go:22-79
 *   checkMode             internal/lossy/decode_frame.go:6-19
 *   doFilter              internal/lossy/decode_frame.go:293-342
 *   parseFrame ordering   internal/lossy/decode.go:532-560
 * kScan: internal/lossy/decode.go:575-580.
 */
#include <string.h>
#include <stdlib.h>
#include "oracle.h"

#define BPS OR_BPS

static int check_mode(int mbx, int mby, int mode) { /* decode_frame.go:6 */
  if (mode == 0) {
    if (mbx == 0) return mby == 0 ? 6 : 5;
    if (mby == 0) return 4;
  }
  return mode;
}

static void do_transform(uint32_t bits, const int16_t* src, uint8_t* dst) { /* :22 */
  switch (bits >> 30) {
    case 3: or_transform(src, dst, 0); break;
    case 2: or_transform_ac3(src, dst); break;
    case 1: { /* inline DC-only, :31-41 */
      int add = (src[0] + 4) >> 3;
      for (int j = 0; j < 4; j++)
        for (int i = 0; i < 4; i++) dst[i + j * BPS] = (uint8_t)or_clip8b(dst[i + j * BPS] + add);
      break;
    }
    default: break;
  }
}

static void do_uv_transform(uint32_t bits, const int16_t* src, uint8_t* dst) { /* :47 */
  if (!(bits & 0xff)) return;
  if (bits & 0xaa) {
    or_transform_uv(src, dst);
    return;
  }
  static const int offs[4] = {0, 4, 4 * BPS, 4 * BPS + 4};
  for (int k = 0; k < 4; k++) {
    const int16_t* s = src + 16 * k;
    if (!s[0]) continue;
    int add = (s[0] + 4) >> 3; /* doTransformDCBlock :70 */
    for (int j = 0; j < 4; j++)
      for (int i = 0; i < 4; i++) dst[offs[k] + i + j * BPS] = (uint8_t)or_clip8b(dst[offs[k] + i + j * BPS] + add);
  }
}

static const int k_scan[16] = {0, 4, 8, 12, 0 + 4 * BPS, 4 + 4 * BPS, 8 + 4 * BPS, 12 + 4 * BPS,
                               0 + 8 * BPS, 4 + 8 * BPS, 8 + 8 * BPS, 12 + 8 * BPS,
                               0 + 12 * BPS, 4 + 12 * BPS, 8 + 12 * BPS, 12 + 12 * BPS};

typedef struct { uint8_t y[16], u[8], v[8]; } top_t; /* TopSamples decode.go:128-132 */

/* one MB row of reconstructRow; buf is the decoder's yuvB work buffer */
static void reconstruct_row(const or_mb_info* mbrow, const int16_t* coeffs, int mby, int mbw, int mbh,
                            uint8_t* buf, top_t* yuv_t, uint8_t* Y, uint8_t* U, uint8_t* V) {
  const int yb = OR_YOFF, ub = OR_UOFF, vb = OR_VOFF;
  for (int j = 0; j < 16; j++) buf[yb + j * BPS - 1] = 129;
  for (int j = 0; j < 8; j++) { buf[ub + j * BPS - 1] = 129; buf[vb + j * BPS - 1] = 129; }
  if (mby > 0) {
    buf[yb - 1 - BPS] = buf[ub - 1 - BPS] = buf[vb - 1 - BPS] = 129;
  } else {
    memset(buf + yb - BPS - 1, 127, 16 + 4 + 1);
    memset(buf + ub - BPS - 1, 127, 8 + 1);
    memset(buf + vb - BPS - 1, 127, 8 + 1);
  }
  const int ys = 16 * mbw, uvs = 8 * mbw;
  for (int mbx = 0; mbx < mbw; mbx++) {
    const or_mb_info* b = &mbrow[mbx];
    const int16_t* co = coeffs + (size_t)mbx * 384;
    if (mbx > 0) { /* rotate left samples, :118-126 */
      for (int j = -1; j < 16; j++) memcpy(buf + yb + j * BPS - 4, buf + yb + j * BPS + 12, 4);
      for (int j = -1; j < 8; j++) {
        memcpy(buf + ub + j * BPS - 4, buf + ub + j * BPS + 4, 4);
        memcpy(buf + vb + j * BPS - 4, buf + vb + j * BPS + 4, 4);
      }
    }
    top_t* top = &yuv_t[mbx];
    uint32_t bits = b->non_zero_y;
    if (mby > 0) {
      memcpy(buf + yb - BPS, top->y, 16);
      memcpy(buf + ub - BPS, top->u, 8);
      memcpy(buf + vb - BPS, top->v, 8);
    }
    if (b->is_i4x4) {
      uint8_t* tr = buf + yb - BPS + 16;
      if (mby > 0) {
        if (mbx >= mbw - 1) memset(tr, top->y[15], 4);
        else memcpy(tr, yuv_t[mbx + 1].y, 4);
      }
      for (int r = 1; r <= 3; r++) memcpy(tr + r * 4 * BPS, tr, 4);
      for (int n = 0; n < 16; n++, bits <<= 2) {
        int off = yb + k_scan[n];
        or_pred_luma4(b->imodes[n], buf, off);
        do_transform(bits, co + n * 16, buf + off);
      }
    } else {
      or_pred_luma16(check_mode(mbx, mby, b->imodes[0]), buf, yb);
      if (bits)
        for (int n = 0; n < 16; n++, bits <<= 2) do_transform(bits, co + n * 16, buf + yb + k_scan[n]);
    }
    int uvm = check_mode(mbx, mby, b->uv_mode);
    or_pred_chroma8(uvm, buf, ub);
    or_pred_chroma8(uvm, buf, vb);
    do_uv_transform(b->non_zero_uv >> 0, co + 16 * 16, buf + ub);
    do_uv_transform(b->non_zero_uv >> 8, co + 20 * 16, buf + vb);
    if (mby < mbh - 1) { /* stash top samples :190-194 */
      memcpy(top->y, buf + yb + 15 * BPS, 16);
      memcpy(top->u, buf + ub + 7 * BPS, 8);
      memcpy(top->v, buf + vb + 7 * BPS, 8);
    }
    uint8_t* yo = Y + (size_t)mby * 16 * ys + mbx * 16;
    uint8_t* uo = U + (size_t)mby * 8 * uvs + mbx * 8;
    uint8_t* vo = V + (size_t)mby * 8 * uvs + mbx * 8;
    for (int j = 0; j < 16; j++) memcpy(yo + (size_t)j * ys, buf + yb + j * BPS, 16);
    for (int j = 0; j < 8; j++) {
      memcpy(uo + (size_t)j * uvs, buf + ub + j * BPS, 8);
      memcpy(vo + (size_t)j * uvs, buf + vb + j * BPS, 8);
    }
  }
}

/* doFilter :293-342 for one macroblock */
static void filter_mb(const or_mb_info* b, int filter_type, int mbx, int mby, int mbw, uint8_t* Y, uint8_t* U,
                      uint8_t* V) {
  int limit = b->f_limit;
  if (limit == 0) return;
  int ilevel = b->f_ilevel, inner = b->f_inner, hev_t = b->hev_thresh;
  int ys = 16 * mbw;
  int yoff = mby * 16 * ys + mbx * 16;
  if (filter_type == 1) {
    if (mbx > 0) or_simple_hfilter16(Y, yoff, ys, limit + 4);
    if (inner) or_simple_hfilter16i(Y, yoff, ys, limit);
    if (mby > 0) or_simple_vfilter16(Y, yoff, ys, limit + 4);
    if (inner) or_simple_vfilter16i(Y, yoff, ys, limit);
  } else {
    int uvs = 8 * mbw;
    int uvoff = mby * 8 * uvs + mbx * 8;
    if (mbx > 0) {
      or_hfilter16(Y, yoff, ys, limit + 4, ilevel, hev_t);
      or_hfilter8(U, V, uvoff, uvoff, uvs, limit + 4, ilevel, hev_t);
    }
    if (inner) {
      or_hfilter16i(Y, yoff, ys, limit, ilevel, hev_t);
      or_hfilter8i(U, V, uvoff, uvoff, uvs, limit, ilevel, hev_t);
    }
    if (mby > 0) {
      or_vfilter16(Y, yoff, ys, limit + 4, ilevel, hev_t);
      or_vfilter8(U, V, uvoff, uvoff, uvs, limit + 4, ilevel, hev_t);
    }
    if (inner) {
      or_vfilter16i(Y, yoff, ys, limit, ilevel, hev_t);
      or_vfilter8i(U, V, uvoff, uvoff, uvs, limit, ilevel, hev_t);
    }
  }
}

static void run_frame(const or_mb_info* mb, const int16_t* coeffs, int filter_type, int mbw, int mbh,
                      uint8_t* Y, uint8_t* U, uint8_t* V, int do_recon, int do_filter) {
  uint8_t buf[OR_YUV_SIZE];
  memset(buf, 0, sizeof(buf));
  top_t* yuv_t = (top_t*)calloc((size_t)mbw, sizeof(top_t));
  for (int mby = 0; mby < mbh; mby++) {
    const or_mb_info* row = mb + (size_t)mby * mbw;
    if (do_recon)
      reconstruct_row(row, coeffs + (size_t)mby * mbw * 384, mby, mbw, mbh, buf, yuv_t, Y, U, V);
    if (do_filter && filter_type > 0)
      for (int mbx = 0; mbx < mbw; mbx++) filter_mb(&row[mbx], filter_type, mbx, mby, mbw, Y, U, V);
  }
  free(yuv_t);
}

void or_decode_reconstruct(const or_mb_info* mb, const int16_t* coeffs, int mbw, int mbh, uint8_t* y,
                           uint8_t* u, uint8_t* v) {
  run_frame(mb, coeffs, 0, mbw, mbh, y, u, v, 1, 0);
}
void or_decode_filter(const or_mb_info* mb, int filter_type, int mbw, int mbh, uint8_t* y, uint8_t* u,
                      uint8_t* v) {
  run_frame(mb, NULL, filter_type, mbw, mbh, y, u, v, 0, 1);
}
void or_decode_frame(const or_mb_info* mb, const int16_t* coeffs, int filter_type, int mbw, int mbh, uint8_t* y,
                     uint8_t* u, uint8_t* v) {
  run_frame(mb, coeffs, filter_type, mbw, mbh, y, u, v, 1, 1);
}
