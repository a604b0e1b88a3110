/* oracle/rescale.c -- TEST INFRASTRUCTURE ONLY (see oracle/oracle.h).
 * C restatement of the reference's row rescaler:
 *   internal/dsp/rescale.go   multFix :44, multFixFloor :50, rescalerFrac :55,
 *                             RescalerInit :63-105, RescalerImportRow :110-124,
 *                             rescalerImportRowExpand :128-153,
 *                             rescalerImportRowShrink :157-181,
 *                             RescalerExportRow :185-199,
 *                             rescalerExportRowExpand :203-231,
 *                             rescalerExportRowShrink :235-257
 * The Go type keeps libwebp's field names but not all of libwebp's arithmetic
 * (no x_add-1 adjustments, FYScale only in expand mode); the Go code wins for
 * parity, so this follows it statement by statement, int32/uint32 wrap-around
 * included.  The reference has no tests and no callers for this file: parity
 * is pinned by properties only (identity size is the identity, constant
 * planes stay constant under shrink) -- "parity pinned by properties".
 *
 * or_rescale_plane() is the plane driver the reference leaves to its caller
 * (libwebp's WebPRescalerImport/Export loop): import a source row while the
 * rescaler needs one, otherwise export a destination row, until every
 * destination row is out or the source is exhausted. */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define RFIX 32
#define ONE ((uint64_t)1 << RFIX)

static uint32_t mult_fix(uint32_t x, uint32_t y) {
  return (uint32_t)(((uint64_t)x * y + ((uint64_t)1 << (RFIX - 1))) >> RFIX);
}
static uint32_t mult_fix_floor(uint32_t x, uint32_t y) { return (uint32_t)(((uint64_t)x * y) >> RFIX); }
static uint32_t rescaler_frac(int64_t x, int64_t y) {
  if (y == 0) return 0;
  return (uint32_t)(((uint64_t)x << RFIX) / (uint64_t)y);
}

void or_rescaler_init(or_rescaler* r, int sw, int sh, int dw, int dh) {
  memset(r, 0, sizeof(*r));
  r->src_width = sw;
  r->src_height = sh;
  r->dst_width = dw;
  r->dst_height = dh;
  r->x_expand = dw > sw;
  r->y_expand = dh > sh;
  r->frow = (int32_t*)calloc(dw > 0 ? dw : 1, sizeof(int32_t));
  r->irow = (int32_t*)calloc(dw > 0 ? dw : 1, sizeof(int32_t));
  r->x_add = sw;
  r->x_sub = dw;
  r->y_add = sh;
  r->y_sub = dh;
  r->y_accum = r->y_expand ? r->y_sub : r->y_add;
  if (!r->x_expand && r->x_sub > 0) r->fx_scale = rescaler_frac(1, r->x_sub);
  if (r->y_expand && r->y_sub > 0) r->fy_scale = rescaler_frac(1, r->y_sub);
  if (!r->y_expand && r->x_add > 0 && r->y_add > 0) {
    const uint64_t ratio = ((uint64_t)dh << RFIX) / ((uint64_t)r->x_add * (uint64_t)r->y_add);
    r->fxy_scale = ratio != (uint64_t)(uint32_t)ratio ? 0 : (uint32_t)ratio;
  }
}

void or_rescaler_free(or_rescaler* r) {
  free(r->frow);
  free(r->irow);
  r->frow = r->irow = NULL;
}

/* rescalerImportRowExpand (:128-153); int32 products wrap like Go's */
static void import_row_expand(or_rescaler* r, const uint8_t* src) {
  int x_in = 0, x_out = 0;
  int64_t accum = r->x_add;
  int32_t left = src[0];
  int32_t right = r->src_width > 1 ? src[1] : left;
  x_in = 1;
  for (;;) {
    r->frow[x_out] = (int32_t)((uint32_t)right * (uint32_t)r->x_add +
                               (uint32_t)(left - right) * (uint32_t)(int32_t)accum);
    x_out++;
    if (x_out >= r->dst_width) break;
    accum -= r->x_sub;
    if (accum < 0) {
      left = right;
      x_in++;
      if (x_in < r->src_width) right = src[x_in];
      accum += r->x_add;
    }
  }
}

/* rescalerImportRowShrink (:157-181) */
static void import_row_shrink(or_rescaler* r, const uint8_t* src) {
  int x_in = 0, x_out = 0;
  uint32_t sum = 0;
  int64_t accum = 0;
  while (x_out < r->dst_width) {
    uint32_t base = 0;
    accum += r->x_add;
    while (accum > 0) {
      accum -= r->x_sub;
      if (x_in < r->src_width) base = src[x_in];
      sum += base;
      x_in++;
    }
    const uint32_t frac = base * (uint32_t)(-accum);
    r->frow[x_out] = (int32_t)(sum * (uint32_t)r->x_sub - frac);
    sum = mult_fix(frac, r->fx_scale);
    x_out++;
  }
}

void or_rescaler_import_row(or_rescaler* r, const uint8_t* src) {
  if (r->x_expand)
    import_row_expand(r, src);
  else
    import_row_shrink(r, src);
  if (!r->y_expand)
    for (int x = 0; x < r->dst_width; x++) r->irow[x] = (int32_t)((uint32_t)r->irow[x] + (uint32_t)r->frow[x]);
  r->src_y++;
  r->y_accum -= r->y_sub;
}

static uint8_t clip_u(uint32_t v) { return (uint8_t)(v > 255 ? 255 : v); }

int or_rescaler_export_row(or_rescaler* r, uint8_t* dst) {
  if (r->y_accum > 0) return 0;
  if (r->y_expand) {
    /* rescalerExportRowExpand (:203-231) */
    if (r->y_accum == 0) {
      for (int x = 0; x < r->dst_width; x++) dst[x] = clip_u(mult_fix((uint32_t)r->frow[x], r->fy_scale));
    } else {
      const uint32_t b = rescaler_frac(-r->y_accum, r->y_sub);
      const uint32_t a = (uint32_t)(ONE - (uint64_t)b);
      for (int x = 0; x < r->dst_width; x++) {
        const uint64_t i = (uint64_t)a * (uint32_t)r->frow[x] + (uint64_t)b * (uint32_t)r->irow[x];
        const uint32_t j = (uint32_t)((i + ((uint64_t)1 << (RFIX - 1))) >> RFIX);
        dst[x] = clip_u(mult_fix(j, r->fy_scale));
      }
    }
    memcpy(r->irow, r->frow, sizeof(int32_t) * r->dst_width);
  } else {
    /* rescalerExportRowShrink (:235-257) */
    const uint32_t yscale = r->fy_scale * (uint32_t)(-r->y_accum);
    if (yscale != 0) {
      for (int x = 0; x < r->dst_width; x++) {
        const uint32_t frac = mult_fix_floor((uint32_t)r->frow[x], yscale);
        dst[x] = clip_u(mult_fix((uint32_t)r->irow[x] - frac, r->fxy_scale));
        r->irow[x] = (int32_t)frac;
      }
    } else {
      for (int x = 0; x < r->dst_width; x++) {
        dst[x] = clip_u(mult_fix((uint32_t)r->irow[x], r->fxy_scale));
        r->irow[x] = 0;
      }
    }
  }
  r->y_accum += r->y_add;
  r->dst_y++;
  return 1;
}

int or_rescale_plane(const uint8_t* src, int sw, int sh, int src_stride, uint8_t* dst, int dw, int dh,
                     int dst_stride) {
  or_rescaler r;
  or_rescaler_init(&r, sw, sh, dw, dh);
  while (r.dst_y < dh) {
    if (r.y_accum > 0) { /* RescalerNeedsSrcRow */
      if (r.src_y >= sh) break;
      or_rescaler_import_row(&r, src + (size_t)r.src_y * src_stride);
    } else {
      or_rescaler_export_row(&r, dst + (size_t)r.dst_y * dst_stride);
    }
  }
  const int rows = r.dst_y;
  or_rescaler_free(&r);
  return rows;
}
