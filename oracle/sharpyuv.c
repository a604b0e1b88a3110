/* sharpyuv.c -- TEST INFRASTRUCTURE ONLY.  C restatement of the reference's
 * SharpYUV RGB -> YUV420 conversion, sRGB transfer:
 *
 *   sharpyuv/sharpyuv.go:39-64   Convert
 *                        :68-115  convertStandard (SharpEnabled = false)
 *                        :140-168 getPrecisionShift, rgbToGray, scaleDown
 *                        :170-269 convertSharp (import, 4 Gauss-Seidel
 *                                 iterations with early exit, final matrix)
 *                        :271-432 importOneRow, storeGray, updateW,
 *                                 updateChroma, filter2, interpolateTwoRows,
 *                                 sharpYUVUpdateY/RGB, convertWRGBToYUV
 *   sharpyuv/gamma.go:48-123     initGammaTables, shiftVal,
 *                                 fixedPointInterpolation, to/fromLinearSrgb
 *   sharpyuv/csp.go:62-90        conversion matrices
 *
 * The gamma tables come from math.Pow in the reference; here libm pow (the
 * values are rounded to integers, so an ulp difference could only matter at
 * a rounding boundary; the tables are exported so tests can compare).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define YUV_FIX 16
#define YUV_HALF (1 << (YUV_FIX - 1))
#define G2L_BITS 10
#define G2L_SIZE (1 << G2L_BITS)
#define L2G_BITS 9
#define L2G_SIZE (1 << L2G_BITS)
#define G2L_VALUE_BITS 16

static uint32_t g2l[G2L_SIZE + 2], l2g[L2G_SIZE + 2];
static int tables_ready = 0;

/* initGammaTables (gamma.go:48-88) */
static void init_tables(void) {
  if (tables_ready) return;
  const double a = 0.09929682680944, thresh = 0.018053968510807;
  const double gamma_f = 1.0 / 0.45, final_scale = (double)(1u << G2L_VALUE_BITS);
  const double norm = 1.0 / (double)G2L_SIZE, a_rec = 1.0 / (1.0 + a);
  for (int v = 0; v <= G2L_SIZE; v++) {
    const double g = norm * (double)v;
    const double value = g <= thresh * 4.5 ? g / 4.5 : pow(a_rec * (g + a), gamma_f);
    g2l[v] = (uint32_t)(value * final_scale + 0.5);
  }
  g2l[G2L_SIZE + 1] = g2l[G2L_SIZE];
  const double scale = 1.0 / (double)L2G_SIZE;
  for (int v = 0; v <= L2G_SIZE; v++) {
    const double g = scale * (double)v;
    const double value = g <= thresh ? 4.5 * g : (1.0 + a) * pow(g, 1.0 / gamma_f) - a;
    l2g[v] = (uint32_t)(final_scale * value + 0.5);
  }
  l2g[L2G_SIZE + 1] = l2g[L2G_SIZE];
  tables_ready = 1;
}

void or_sharpyuv_tables(uint32_t* g2l_out, uint32_t* l2g_out) {
  init_tables();
  memcpy(g2l_out, g2l, sizeof(g2l));
  memcpy(l2g_out, l2g, sizeof(l2g));
}

static int shift_val(int v, int shift) { return shift >= 0 ? v << shift : v >> -shift; }

/* fixedPointInterpolation (gamma.go:97-109) */
static uint32_t fp_interp(int v, const uint32_t* tab, int pos_shr, int val_shift) {
  const int pos = shift_val(v, -pos_shr);
  const uint32_t x = (uint32_t)(v - shift_val(pos, pos_shr));
  const uint32_t v0 = (uint32_t)shift_val((int)tab[pos], val_shift);
  const uint32_t v1 = (uint32_t)shift_val((int)tab[pos + 1], val_shift);
  const uint32_t v2 = (v1 - v0) * x;
  const int half = pos_shr > 0 ? 1 << (pos_shr - 1) : 0;
  return v0 + ((v2 + (uint32_t)half) >> pos_shr);
}
/* toLinearSrgb / fromLinearSrgb (gamma.go:111-123) */
static uint32_t to_linear(uint16_t v, int bit_depth) {
  const int shift = G2L_BITS - bit_depth;
  if (shift > 0) return g2l[(int)v << shift];
  return fp_interp((int)v, g2l, -shift, 0);
}
static uint16_t from_linear(uint32_t value, int bit_depth) {
  return (uint16_t)fp_interp((int)value, l2g, G2L_VALUE_BITS - L2G_BITS, bit_depth - G2L_VALUE_BITS);
}

static int rgb_to_gray(int64_t r, int64_t g, int64_t b) {
  return (int)((13933 * r + 46871 * g + 4732 * b + YUV_HALF) >> YUV_FIX);
}
static uint32_t scale_down(uint16_t a, uint16_t b, uint16_t c, uint16_t d, int bd) {
  const uint32_t la = to_linear(a, bd), lb = to_linear(b, bd), lc = to_linear(c, bd), ld = to_linear(d, bd);
  return from_linear((la + lb + lc + ld + 2) >> 2, bd);
}
static uint16_t clip_bd(int y, int bd) {
  const int mx = (1 << bd) - 1;
  return (uint16_t)(y < 0 ? 0 : (y > mx ? mx : y));
}
static uint8_t clip_u8(int32_t v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

static void import_row(const uint8_t* rgb, int row, int stride, int pic_w, int w, int sfix, uint16_t* dst) {
  const uint8_t* p = rgb + (size_t)row * stride;
  for (int i = 0; i < pic_w; i++) {
    dst[i] = (uint16_t)shift_val(p[3 * i + 0], sfix);
    dst[i + w] = (uint16_t)shift_val(p[3 * i + 1], sfix);
    dst[i + 2 * w] = (uint16_t)shift_val(p[3 * i + 2], sfix);
  }
  if (pic_w < w) {
    dst[pic_w] = dst[pic_w - 1];
    dst[pic_w + w] = dst[pic_w + w - 1];
    dst[pic_w + 2 * w] = dst[pic_w + 2 * w - 1];
  }
}
static void store_gray(const uint16_t* src, uint16_t* y, int w) {
  for (int i = 0; i < w; i++) y[i] = (uint16_t)rgb_to_gray(src[i], src[i + w], src[i + 2 * w]);
}
static void update_w(const uint16_t* src, uint16_t* dst, int w, int bd) {
  for (int i = 0; i < w; i++) {
    const uint32_t r = to_linear(src[i], bd), g = to_linear(src[i + w], bd), b = to_linear(src[i + 2 * w], bd);
    dst[i] = from_linear((uint32_t)rgb_to_gray(r, g, b), bd);
  }
}
static void update_chroma(const uint16_t* s1, const uint16_t* s2, int16_t* dst, int uvw, int bd) {
  const int w = uvw * 2;
  for (int i = 0; i < uvw; i++) {
    const int i2 = 2 * i;
    const int r = (int)scale_down(s1[i2], s1[i2 + 1], s2[i2], s2[i2 + 1], bd);
    const int g = (int)scale_down(s1[i2 + w], s1[i2 + w + 1], s2[i2 + w], s2[i2 + w + 1], bd);
    const int b = (int)scale_down(s1[i2 + 2 * w], s1[i2 + 2 * w + 1], s2[i2 + 2 * w], s2[i2 + 2 * w + 1], bd);
    const int gray = rgb_to_gray(r, g, b);
    dst[i] = (int16_t)(r - gray);
    dst[i + uvw] = (int16_t)(g - gray);
    dst[i + 2 * uvw] = (int16_t)(b - gray);
  }
}
static uint16_t filter2(int a, int b, int w0, int bd) { return clip_bd(((a * 3 + b + 2) >> 2) + w0, bd); }
static void interpolate_two_rows(const uint16_t* best_y, const int16_t* prev, const int16_t* cur, const int16_t* next,
                                 int w, uint16_t* out1, uint16_t* out2, int bd) {
  const int uvw = w >> 1, flen = (w - 1) >> 1;
  for (int k = 0; k < 3; k++) {
    const int ku = k * uvw, kw = k * w;
    out1[kw] = filter2(cur[ku], prev[ku], best_y[0], bd);
    out2[kw] = filter2(cur[ku], next[ku], best_y[w], bd);
    for (int i = 0; i < flen; i++) {
      const int a0 = cur[ku + i], a1 = cur[ku + i + 1], b0 = prev[ku + i], b1 = prev[ku + i + 1];
      const int v0 = (a0 * 9 + a1 * 3 + b0 * 3 + b1 + 8) >> 4;
      const int v1 = (a1 * 9 + a0 * 3 + b1 * 3 + b0 + 8) >> 4;
      out1[kw + 2 * i + 1] = clip_bd(best_y[2 * i + 1] + v0, bd);
      out1[kw + 2 * i + 2] = clip_bd(best_y[2 * i + 2] + v1, bd);
      const int n0 = next[ku + i], n1 = next[ku + i + 1];
      const int nv0 = (a0 * 9 + a1 * 3 + n0 * 3 + n1 + 8) >> 4;
      const int nv1 = (a1 * 9 + a0 * 3 + n1 * 3 + n0 + 8) >> 4;
      out2[kw + 2 * i + 1] = clip_bd(best_y[w + 2 * i + 1] + nv0, bd);
      out2[kw + 2 * i + 2] = clip_bd(best_y[w + 2 * i + 2] + nv1, bd);
    }
    if ((w & 1) == 0) {
      out1[kw + w - 1] = filter2(cur[ku + uvw - 1], prev[ku + uvw - 1], best_y[w - 1], bd);
      out2[kw + w - 1] = filter2(cur[ku + uvw - 1], next[ku + uvw - 1], best_y[2 * w - 1], bd);
    }
  }
}
static uint64_t update_y(const uint16_t* target, const uint16_t* src, uint16_t* dst, int len, int bd) {
  uint64_t diff = 0;
  const int max_y = (1 << bd) - 1;
  for (int i = 0; i < len; i++) {
    const int d = (int)target[i] - (int)src[i];
    const int ny = (int)dst[i] + d;
    dst[i] = (uint16_t)(ny < 0 ? 0 : (ny > max_y ? max_y : ny));
    diff += (uint64_t)(d < 0 ? -d : d);
  }
  return diff;
}
static void update_rgb(const int16_t* target, const int16_t* src, int16_t* dst, int len) {
  for (int i = 0; i < len; i++) {
    const int16_t d = (int16_t)(target[i] - src[i]); /* int16 arithmetic wraps, as in Go */
    dst[i] = (int16_t)(dst[i] + d);
  }
}

/* matrix: rgb_to_y[4], rgb_to_u[4], rgb_to_v[4] (csp.go ConversionMatrix) */
static void convert_wrgb_to_yuv(const uint16_t* best_y, const int16_t* best_uv, uint8_t* y, int y_stride, uint8_t* u,
                                uint8_t* v, int uv_stride, int width, int height, int w, int uvw, int uvh, int sfix,
                                const int32_t* m) {
  const int64_t rounder = (int64_t)1 << (YUV_FIX + sfix - 1);
  const int64_t y_off = shift_val(m[3], sfix), u_off = shift_val(m[7], sfix), v_off = shift_val(m[11], sfix);
  for (int j = 0; j < height; j++)
    for (int i = 0; i < width; i++) {
      const int uvi = (j / 2) * 3 * uvw + (i >> 1);
      const int64_t wv = best_y[j * w + i];
      const int64_t r = best_uv[uvi] + wv, g = best_uv[uvi + uvw] + wv, b = best_uv[uvi + 2 * uvw] + wv;
      const int64_t yv = (int64_t)m[0] * r + (int64_t)m[1] * g + (int64_t)m[2] * b + y_off + rounder;
      y[(size_t)j * y_stride + i] = clip_u8((int32_t)(yv >> (YUV_FIX + sfix)));
    }
  for (int j = 0; j < uvh; j++)
    for (int i = 0; i < uvw; i++) {
      const int uvi = j * 3 * uvw + i;
      const int64_t r = best_uv[uvi], g = best_uv[uvi + uvw], b = best_uv[uvi + 2 * uvw];
      const int64_t uv = (int64_t)m[4] * r + (int64_t)m[5] * g + (int64_t)m[6] * b + u_off + rounder;
      const int64_t vv = (int64_t)m[8] * r + (int64_t)m[9] * g + (int64_t)m[10] * b + v_off + rounder;
      u[(size_t)j * uv_stride + i] = clip_u8((int32_t)(uv >> (YUV_FIX + sfix)));
      v[(size_t)j * uv_stride + i] = clip_u8((int32_t)(vv >> (YUV_FIX + sfix)));
    }
}

/* convertSharp (sharpyuv.go:170-269).  Returns the number of iterations run. */
int or_sharpyuv_convert(const uint8_t* rgb, int width, int height, int rgb_stride, uint8_t* y, int y_stride,
                        uint8_t* u, uint8_t* v, int uv_stride, const int32_t* matrix) {
  init_tables();
  const int w = (width + 1) & ~1, h = (height + 1) & ~1;
  const int uvw = w >> 1, uvh = h >> 1, sfix = 2, bd = 8 + sfix;
  uint16_t* tmp1 = malloc(sizeof(uint16_t) * 3 * w);
  uint16_t* tmp2 = malloc(sizeof(uint16_t) * 3 * w);
  uint16_t* best_y = malloc(sizeof(uint16_t) * w * h);
  uint16_t* target_y = malloc(sizeof(uint16_t) * w * h);
  int16_t* best_uv = malloc(sizeof(int16_t) * 3 * uvw * uvh);
  int16_t* target_uv = malloc(sizeof(int16_t) * 3 * uvw * uvh);
  uint16_t* best_rgb_y = malloc(sizeof(uint16_t) * 2 * w);
  int16_t* best_rgb_uv = malloc(sizeof(int16_t) * 3 * uvw);
  for (int j = 0; j < height; j += 2) {
    const int last = j == height - 1;
    import_row(rgb, j, rgb_stride, width, w, sfix, tmp1);
    if (!last) import_row(rgb, j + 1, rgb_stride, width, w, sfix, tmp2);
    else memcpy(tmp2, tmp1, sizeof(uint16_t) * 3 * w);
    const int boff = (j / 2) * 2 * w, uoff = (j / 2) * 3 * uvw;
    store_gray(tmp1, best_y + boff, w);
    store_gray(tmp2, best_y + boff + w, w);
    update_w(tmp1, target_y + boff, w, bd);
    update_w(tmp2, target_y + boff + w, w, bd);
    update_chroma(tmp1, tmp2, target_uv + uoff, uvw, bd);
    memcpy(best_uv + uoff, target_uv + uoff, sizeof(int16_t) * 3 * uvw);
  }
  const uint64_t thr = (uint64_t)3 * w * h;
  uint64_t prev_sum = ~(uint64_t)0;
  int iters = 0;
  for (int it = 0; it < 4; it++) {
    uint64_t sum = 0;
    for (int j = 0; j < h; j += 2) {
      const int ju = j / 2;
      const int cur = ju * 3 * uvw;
      const int prev = ju > 0 ? (ju - 1) * 3 * uvw : cur;
      const int next = j < h - 2 ? (ju + 1) * 3 * uvw : cur;
      interpolate_two_rows(best_y + j * w, best_uv + prev, best_uv + cur, best_uv + next, w, tmp1, tmp2, bd);
      update_w(tmp1, best_rgb_y, w, bd);
      update_w(tmp2, best_rgb_y + w, w, bd);
      update_chroma(tmp1, tmp2, best_rgb_uv, uvw, bd);
      sum += update_y(target_y + j * w, best_rgb_y, best_y + j * w, 2 * w, bd);
      update_rgb(target_uv + ju * 3 * uvw, best_rgb_uv, best_uv + cur, 3 * uvw);
    }
    iters++;
    if (it > 0 && (sum < thr || sum > prev_sum)) break;
    prev_sum = sum;
  }
  convert_wrgb_to_yuv(best_y, best_uv, y, y_stride, u, v, uv_stride, width, height, w, uvw, uvh, sfix, matrix);
  free(tmp1);
  free(tmp2);
  free(best_y);
  free(target_y);
  free(best_uv);
  free(target_uv);
  free(best_rgb_y);
  free(best_rgb_uv);
  return iters;
}
